"""docs/ENV.md lists runtime switches: every variable it names must still be read somewhere in
the package or the bench (a renamed or removed switch makes the doc lie)."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_every_documented_switch_exists():
    doc = (ROOT / "docs" / "ENV.md").read_text()
    names = set(re.findall(r"HIPZAP_[A-Z0-9_]+", doc))
    assert names, "no switches documented?"
    code = "".join(p.read_text(errors="ignore") for ext in ("*.py", "*.cpp", "*.hip", "*.h")
                   for p in (ROOT / "hipzap").rglob(ext))
    code += (ROOT / "bench.py").read_text()
    # prefixes documented with a wildcard (HIPZAP_CHAIN_*) match any variable they start
    missing = sorted(n for n in names if n not in code and not (n.endswith("_") and n in code))
    assert not missing, missing
