"""The torch-free checkpoint path on the CPU: the weights-only ``torch.save`` reader
(hipzap/pthreader.py) against torch.load, its refusal of anything outside the allowlist, the numpy
packer (engine/nppack.py) bitwise against the torch packer, and a weightless plan template
(engine/plan.py export_template) placing every packed parameter exactly where the full plan image
exported from the same checkpoint has it (the device packer writes those slots on the GPU:
tests/test_pth_lite_gpu.py)."""
import base64
import io
import os
import pickle
import sys
import zipfile

import numpy as np
import pytest
import torch

from hipzap import pthreader
from hipzap.engine import nppack
from hipzap.models.resnet import pack_resnet, randomize_bn, resnet18, resnet50


def _ckpt(tmp_path, mk, name="m.pth"):
    torch.manual_seed(0)
    m = randomize_bn(mk()).eval()
    p = str(tmp_path / name)
    torch.save(m.state_dict(), p)
    return p, m.state_dict()


def test_reader_matches_torch_load(tmp_path):
    p, _ = _ckpt(tmp_path, resnet18)
    ref = torch.load(p, weights_only=True)
    sd = pthreader.load_state_dict(p)
    assert list(sd) == list(ref)
    for k, v in ref.items():
        assert sd[k].shape == tuple(v.shape) and np.array_equal(sd[k], v.numpy()), k
    x = {"bf": torch.randn(5, 3).bfloat16(), "h": torch.randn(4).half(), "sc": torch.tensor(3.5), "t": torch.randn(6, 4),
         "i": torch.arange(7), "p": torch.nn.Parameter(torch.randn(3))}
    x["view"], x["tr"], x["tied"] = x["t"][2:, 1:3], x["t"].t(), x["t"]
    torch.save(x, tmp_path / "x.pth")
    y = pthreader.load_state_dict(str(tmp_path / "x.pth"))
    assert np.array_equal(y["bf"].to_float32(), x["bf"].float().numpy())
    for k in ("h", "sc", "t", "i", "p", "view", "tr", "tied"):
        assert np.array_equal(y[k], x[k].detach().numpy()), k
    refs = pthreader.scan(str(tmp_path / "x.pth"))
    assert refs["tied"].storage is refs["t"].storage and refs["view"].offset == 2 * 4 + 1
    assert refs["t"].is_contiguous() and not refs["tr"].is_contiguous() and not refs["view"].is_contiguous()


def test_reader_refuses_non_allowlisted_globals(tmp_path):
    """A data.pkl that names any other global (here os.system) is refused before anything runs."""
    marker = tmp_path / "pwned"

    class Evil:
        def __reduce__(self):
            return os.system, (f"touch {marker}",)

    buf = io.BytesIO()
    pickle.dump({"w": Evil()}, buf, protocol=2)
    p = tmp_path / "evil.pth"
    with zipfile.ZipFile(p, "w", zipfile.ZIP_STORED) as z:
        z.writestr("evil/data.pkl", buf.getvalue())
        z.writestr("evil/byteorder", "little")
    with pytest.raises(pickle.UnpicklingError, match="not allowed"):
        pthreader.load_state_dict(str(p))
    with pytest.raises(pickle.UnpicklingError):
        pthreader.scan(str(p))
    assert not marker.exists()


def test_scan_needs_no_numpy_or_torch(tmp_path):
    p, _ = _ckpt(tmp_path, resnet18)
    code = (f"import sys; from hipzap import pthreader, lite; from hipzap.engine import nppack; "
            f"r = pthreader.scan({p!r}); print(nppack.infer_resnet(r), 'numpy' in sys.modules, 'torch' in sys.modules)")
    import subprocess
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["('resnet18',", "1000)", "False", "False"]


@pytest.mark.parametrize("mk", [resnet18, resnet50])
def test_numpy_pack_is_bitwise_the_torch_pack(tmp_path, mk):
    p, sd = _ckpt(tmp_path, mk)
    P = pack_resnet(torch.load(p, weights_only=True))
    Q = nppack.pack_resnet(pthreader.load_state_dict(p))
    assert set(P) == set(Q)
    for k, pc in P.items():
        assert np.array_equal(pc.wf.view(torch.int16).numpy().view(np.uint16), Q[k]["wf"]), k
        assert np.array_equal(pc.bias.numpy(), Q[k]["bias"]), k


def test_template_places_every_parameter_like_the_plan_image(tmp_path):
    from hipzap.engine.plan import HEADER, export_from_checkpoint, export_template
    from hipzap.lite import read_meta
    p, _ = _ckpt(tmp_path, resnet18)
    plan = export_from_checkpoint("resnet18", p, str(tmp_path / "m.hzplan"))
    tmpl = export_template("resnet18", 1000, 1, 1, True, str(tmp_path / "r18.hztmpl"))
    pm, tm = read_meta(plan), read_meta(tmpl)
    assert tm["weightless"] and os.path.getsize(tmpl) < 1 << 20 and tm["blob_bytes"] == pm["blob_bytes"]
    with open(plan, "rb") as f:
        hdr = HEADER.unpack(f.read(HEADER.size))
        f.seek(hdr[8])
        blob = f.read(hdr[9])
    Q = nppack.pack_resnet(pthreader.load_state_dict(p))
    mine = bytearray(tm["blob_bytes"])
    for slot, (off, nb) in tm["blob_map"].items():
        name, field = slot.split("/")
        data = Q[name][field].tobytes()
        assert len(data) == nb, slot
        mine[off: off + nb] = data
    for off, b64 in tm["blob_consts"]:
        data = base64.b64decode(b64)
        mine[off: off + len(data)] = data
    assert bytes(mine) == blob
    # the recipe covers every packed parameter with its checkpoint sources
    assert set(tm["pack"]) == set(Q) and tm["pack"]["fc"]["kind"] == "linear" and tm["pack"]["conv1"]["cin_p"] == 8


def _forged(tmp_path, off, size, stride, numel=16, name="forged.pth"):
    """A torch.save-shaped archive whose one tensor view has the given geometry (written with the
    real torch._utils rebuild global and storage marker, so only the geometry is hostile)."""
    from collections import OrderedDict

    class _S:
        pass

    class _T:
        def __reduce__(self):
            return torch._utils._rebuild_tensor_v2, (_S(), off, size, stride, False, OrderedDict())

    class _P(pickle.Pickler):
        def persistent_id(self, obj):
            return ("storage", torch.FloatStorage, "0", "cpu", numel) if isinstance(obj, _S) else None

    buf = io.BytesIO()
    _P(buf, protocol=2).dump({"w": _T()})
    p = tmp_path / name
    with zipfile.ZipFile(p, "w", zipfile.ZIP_STORED) as z:
        z.writestr("f/data.pkl", buf.getvalue())
        z.writestr("f/byteorder", "little")
        z.writestr("f/data/0", np.arange(16, dtype=np.float32).tobytes())
    return str(p)


@pytest.mark.parametrize("off,size,stride", [(-4, (4,), (1,)), (0, (4,), (-1,)), (8, (2, 2), (-4, 1)), (0, (-1,), (1,)),
                                             (12, (8,), (1,)), (16, (), ())])
def test_reader_refuses_views_outside_their_record(tmp_path, off, size, stride):
    """Negative offsets / strides / sizes and views past the record would address bytes outside
    the storage (numpy as_strided on the host, the device packer's staging pointer on the GPU):
    refused in both modes, before any array or pointer is formed."""
    p = _forged(tmp_path, off, size, stride)
    with pytest.raises(pickle.UnpicklingError):
        pthreader.load_state_dict(p)
    with pytest.raises(pickle.UnpicklingError):
        pthreader.scan(p)


def test_reader_accepts_forged_but_valid_view(tmp_path):
    p = _forged(tmp_path, 4, (2, 3), (3, 1))
    assert np.array_equal(pthreader.load_state_dict(p)["w"], np.arange(4, 10, dtype=np.float32).reshape(2, 3))
    r = pthreader.scan(p)["w"]
    assert r.offset == 4 and r.shape == (2, 3) and r.is_contiguous()


def test_reader_storage_marker_is_immutable(tmp_path):
    """A BUILD opcode on a storage dtype marker (to rewrite its item size / dtype before a
    persistent id uses it) fails instead of changing what the record is read as."""
    for state in (b"}X\x05\x00\x00\x00dtypeX\x07\x00\x00\x00float64sb.",
                  b"N}X\x04\x00\x00\x00nameX\r\x00\x00\x00DoubleStorages\x86b."):
        p = tmp_path / "m.pth"
        with zipfile.ZipFile(p, "w", zipfile.ZIP_STORED) as z:
            z.writestr("m/data.pkl", b"\x80\x02ctorch\nFloatStorage\n" + state)
        with pytest.raises((pickle.UnpicklingError, AttributeError)):
            pthreader.load_state_dict(str(p))


def test_built_templates_match_the_current_code():
    """A weightless plan template is valid only for the lowering code that wrote it (lite.code_stamp
    over engine/, models/, ops/, tuning/): templates that exist in the tree must carry the current
    stamp, else the torch-free .pth cold start refuses them (rebuild: python -m hipzap.build
    --templates, which __graft_entry__.build() runs)."""
    from hipzap import lite
    for model in ("resnet50", "resnet18"):
        p = lite.template_path(model)
        if not os.path.exists(p):
            continue
        assert lite.read_meta(p).get("code_stamp") == lite.code_stamp(), f"{p} is stale"


def test_upload_stream_only_inside_a_fill():
    """lite.upload_stream() hands a fill_blob callback the plan's upload stream (set by PlanEngine
    around the callback) and is None everywhere else, including other threads during a fill."""
    import threading
    from hipzap import lite
    assert lite.upload_stream() is None
    seen = {}
    lite._fill_tls.stream = 0x1234
    try:
        t = threading.Thread(target=lambda: seen.setdefault("other", lite.upload_stream()))
        t.start()
        t.join()
        seen["self"] = lite.upload_stream()
    finally:
        lite._fill_tls.stream = None
    assert seen == {"other": None, "self": 0x1234}
    assert lite.upload_stream() is None


@pytest.mark.parametrize("key", ["bn1.weight", "layer1.0.bn2.running_var", "fc.bias"])
def test_from_checkpoint_refuses_short_vectors(tmp_path, key):
    """Every BN vector and bias the device packer reads must hold exactly cout elements: a short
    one (which still fits its own storage) is refused before anything is uploaded, instead of the
    pack kernel reading the next staged tensor."""
    from hipzap import lite
    if not os.path.exists(lite.template_path("resnet18")):
        pytest.skip("resnet18 template not built")
    torch.manual_seed(0)
    sd = randomize_bn(resnet18()).eval().state_dict()
    sd[key] = sd[key][:10].clone()
    p = str(tmp_path / "short.pth")
    torch.save(sd, p)
    with pytest.raises(lite.PlanError, match=key.replace(".", r"\.")):
        lite.PlanEngine.from_checkpoint(p)


def _zipfile_index(path):
    with zipfile.ZipFile(path) as zf:
        return {i.filename: (i.compress_type, i.compress_size, i.file_size, i.header_offset, i.flag_bits)
                for i in zf.infolist()}


def test_direct_zip_index_matches_zipfile(tmp_path):
    """The central-directory reader (no zipfile import on the cold-start path) sees exactly what
    zipfile sees: a torch.save archive, and a zip64 archive (> 65535 members: zip64 end records)."""
    import mmap
    p = str(tmp_path / "m.pth")
    torch.save(resnet18().state_dict(), p)
    with open(p, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    assert pthreader._zip_index(mm) == _zipfile_index(p)
    z = str(tmp_path / "many.zip")
    with zipfile.ZipFile(z, "w", allowZip64=True) as zf:
        for i in range(65540):
            zf.writestr(f"a/{i}", b"x")
    with open(z, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        assert mm.rfind(b"PK\x06\x06") > 0  # the zip64 end record is there
    assert pthreader._zip_index(mm) == _zipfile_index(z)
    assert pthreader._zip_index(mmap.mmap(-1, 64)) is None  # not a zip: the caller falls back


def test_reader_without_the_direct_index_is_unchanged(tmp_path, monkeypatch):
    """With the direct index refused (None), the zipfile fallback reads the same state_dict."""
    p = str(tmp_path / "m.pth")
    sd = resnet18().state_dict()
    torch.save(sd, p)
    a = pthreader.load_state_dict(p)
    monkeypatch.setattr(pthreader, "_zip_index", lambda mm: None)
    b = pthreader.load_state_dict(p)
    assert a.keys() == b.keys() and all(np.array_equal(a[k], b[k]) for k in a)
