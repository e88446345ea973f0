"""The in-tree debug library (HIPZAP_DEBUG=1, loaded by tests/test_kcheck_gpu.py on the GPU box)
exports every entry point of the product library: a stale one (built before a new ``hz_*``
function) fails at load time on the GPU box, so catch it here."""
import shutil
import subprocess

import pytest

from hipzap import build as B


def _exports(path) -> set:
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True, check=True).stdout
    return {f[2] for f in (ln.split() for ln in out.splitlines()) if len(f) == 3 and f[1] == "T" and f[2].startswith("hz_")}


@pytest.mark.skipif(shutil.which("nm") is None, reason="needs binutils nm")
def test_debug_library_exports_the_product_entry_points():
    if not B.LIB_DEBUG.exists() or not B.LIB.exists():
        pytest.skip("libraries not built")
    missing = _exports(B.LIB) - _exports(B.LIB_DEBUG)
    assert not missing, f"stale {B.LIB_DEBUG.name}: python -m hipzap.build (missing {sorted(missing)})"
