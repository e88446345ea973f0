"""The torch-free AWD-LSTM path on the CPU (hipzap/lmlite.py, engine/lmcore.py): geometry and
checkpoint rules from the file's shapes alone, the SURVEY §5.4 W_hh key rule, and that the whole
GET /inference cold-start path imports neither torch nor numpy."""
import os
import subprocess
import sys

import pytest
import torch

from hipzap.engine import lmcore
from hipzap.models.awd_lstm import reference_lm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _shapes(sd):
    return {k: tuple(v.shape) for k, v in sd.items()}


def test_geometry_of_reference_dims():
    sd = reference_lm(600).state_dict()
    g = lmcore.geometry(_shapes(sd), tied=True)
    assert (g.V, g.E, g.Ke, g.Vp) == (600, 1000, 1024, 608)
    assert [(ly.H, ly.In, ly.Kh, ly.Kx, ly.R) for ly in g.layers] == [
        (1150, 1000, 1152, 1024, 4608), (1150, 1150, 1152, 1152, 4608), (1000, 1150, 1024, 1152, 4000)]
    assert g.dec_key is None and g.dec_bias_key == "1.decoder.bias"
    assert lmcore.geometry(_shapes(sd), tied=False).dec_key == "1.decoder.weight"


def test_effective_whh_key_rule():
    """module.weight_hh_l0 wins over weight_hh_l0_raw; _raw only when the module key is absent."""
    keys = list(reference_lm(50).state_dict())
    lk = lmcore.layer_keys(keys)
    assert len(lk) == 3 and all(k[1].endswith("module.weight_hh_l0") for k in lk)
    no_mod = [k for k in keys if not k.endswith("module.weight_hh_l0")]
    assert all(k[1].endswith("weight_hh_l0_raw") for k in lmcore.layer_keys(no_mod))


@pytest.mark.parametrize("edit,msg", [
    (lambda s: s.pop("0.encoder.weight"), "no 0.encoder.weight"),
    (lambda s: s.update({"0.rnns.1.module.bias_hh_l0": (7,)}), "inconsistent"),
    (lambda s: s.update({"0.rnns.0.weight_ih_l0_reverse": (4, 4)}), "bidirectional"),
    (lambda s: s.update({"1.decoder.bias": (3,)}), "decoder.bias"),
])
def test_geometry_refusals(edit, msg):
    s = _shapes(reference_lm(64).state_dict())
    edit(s)
    with pytest.raises(ValueError, match=msg):
        lmcore.geometry(s, tied=True)


def test_lm_cold_path_imports_no_torch():
    code = ("import sys; import hipzap.lmlite, hipzap.coldstart, hipzap.serve.text, hipzap.engine.lmcore; "
            "print('torch' in sys.modules, 'numpy' in sys.modules)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["False", "False"]
