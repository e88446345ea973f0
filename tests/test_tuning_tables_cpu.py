"""The shipped tuning tables pick only launch configurations the product library contains: a
table entry naming an experiments-build tile (32x32 LDS tiles cfg 64-77, the MX pipelines and
ping-pong cfgs) would make the lean library refuse the launch at capture time."""
import json
import pathlib

from hipzap.ops import conv as conv_ops
from hipzap.ops import fp8

TABLES = sorted((pathlib.Path(__file__).resolve().parents[1] / "hipzap" / "tuning").glob("*.json"))


def test_tables_exist():
    assert TABLES


def test_tables_name_product_configs_only():
    bad = []
    for t in TABLES:
        for key, val in json.loads(t.read_text()).items():
            cfg = val[0]
            if key.startswith("f8r"):
                if cfg in fp8.MX_EXPERIMENTS or (cfg >= 16 and cfg not in fp8.MX_TILES):
                    bad.append((t.name, key, cfg))
            elif cfg >= 16 and cfg not in conv_ops.LDS_TILES:  # (e.g. the deleted M32 tiles, cfg 64-77)
                bad.append((t.name, key, cfg))
    assert not bad, bad
