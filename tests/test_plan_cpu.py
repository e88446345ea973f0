"""Plan images (engine/plan.py -> csrc/plan.cpp) on the CPU: every pointer of every recorded
launch is relocated, weight relocations land on the same bytes, scalars are preserved, the
header/ABI is what the native loader expects, and the torch-free runtime module imports
without torch."""
import ctypes as C
import json
import os
import subprocess
import sys

import pytest
import torch

from hipzap import _native as N
from hipzap.engine import plan as P
from hipzap.engine.program import ExecContext
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def decode(path):
    raw = open(path, "rb").read()
    f = P.HEADER.unpack_from(raw, 0)
    assert f[0] == P.MAGIC
    hdr = dict(zip(["magic", "version", "abi", "n_ops", "meta_off", "meta_len", "ops_off", "ops_len", "blob_off",
                    "blob_len", "ctx_dev", "ctx_host"], f[:12]))
    meta = json.loads(raw[hdr["meta_off"]: hdr["meta_off"] + hdr["meta_len"]])
    ops, p = [], hdr["ops_off"]
    for _ in range(hdr["n_ops"]):
        t, arg, slot, plen, nrel, _pad = P.OPHDR.unpack_from(raw, p)
        p += P.OPHDR.size
        prm = raw[p: p + plen]
        p += (plen + 7) // 8 * 8
        rels = [P.RELOC.unpack_from(raw, p + i * P.RELOC.size) for i in range(nrel)]
        p += nrel * P.RELOC.size
        ops.append((t, arg, slot, prm, rels))
    assert p == hdr["ops_off"] + hdr["ops_len"]
    blob = raw[hdr["blob_off"]: hdr["blob_off"] + hdr["blob_len"]]
    return hdr, meta, ops, blob


@pytest.fixture(scope="module")
def r18():
    torch.manual_seed(0)
    a = registry.get("resnet18")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack(sd, "cpu")
    return a, params, dict(kw, input_uint8=True)


@pytest.mark.parametrize("zero_copy", ["all", ""])
def test_plan_relocations_cover_every_pointer(tmp_path, r18, zero_copy):
    a, params, kw = r18
    path = str(tmp_path / "r18.hzplan")
    meta = P.export_plan("resnet18", params, kw, path, batch=1, zero_copy=zero_copy)
    hdr, meta2, ops, blob = decode(path)
    assert meta2["n_ops"] == meta["n_ops"] == len(ops)
    assert hdr["version"] == P.VERSION and hdr["abi"] == N.lib().hz_abi_version()
    assert hdr["blob_off"] % P.BLOB_ALIGN == 0
    # re-record the same context: weights are the same tensors, so region-0 relocations must point
    # at byte-identical data; every non-pointer byte must be identical too
    rec = P.PlanRecorder()
    g = a.build_graph(batch=1, **kw)
    ctx = ExecContext(g, params, torch.device("cpu"), None, host_io=True, zero_copy=zero_copy, lib=rec)
    assert len(rec.ops) == len(ops)
    sizes = {0: hdr["blob_len"], 1: hdr["ctx_dev"], 2: hdr["ctx_host"]}
    spans = [(t.untyped_storage().data_ptr(), t.untyped_storage().nbytes())
             for obj in list(params.values()) + list(ctx._keep) for _, t in P._tensors(obj)]

    def left(ptr):  # bytes from ptr to the end of its storage
        return next(b + n - ptr for b, n in spans if b <= ptr < b + n)
    n_w = 0
    for (t, arg, slot, structs), (t2, arg2, slot2, prm, rels) in zip(rec.ops, ops):
        assert (t, arg, slot) == (t2, arg2, slot2)
        raw = b"".join(bytes(s) for s in structs)
        ptr_fields, base = [], 0
        for s in structs:
            ptr_fields += [(base + off, v) for off, v in P._pointer_fields(s)]
            base += C.sizeof(s)
        nonzero = {off: v for off, v in ptr_fields if v}
        assert sorted(off for off, _, _ in rels) == sorted(nonzero), "every non-null pointer relocated"
        for i in range(len(raw)):
            if not any(o <= i < o + 8 for o in nonzero):
                assert raw[i] == prm[i]
        for off, region, roff in rels:
            assert roff < sizes[region]
            if region == 0:
                n = min(16, left(nonzero[off]))
                assert blob[roff: roff + n] == C.string_at(nonzero[off], n)
                n_w += 1
    assert n_w > 20  # ResNet-18: conv weights + biases + head
    ins = meta["inputs"][0]
    assert ins["shape"] == [1, 224, 224, 3] and ins["dtype"] == "uint8"
    assert meta["output"]["dtype"] == "float32" and meta["output"]["shape"][0] == 1
    assert meta["ctx_host_bytes"] >= ins["off"] + ins["bytes"]
    del ctx


def test_plan_blob_is_compact(tmp_path, r18):
    """The blob holds the referenced storages once each, 256-B aligned, and nothing else."""
    a, params, kw = r18
    path = str(tmp_path / "r18.hzplan")
    meta = P.export_plan("resnet18", params, kw, path)
    sts = {t.untyped_storage().data_ptr(): t.untyped_storage().nbytes()
           for obj in params.values() for _, t in P._tensors(obj)}
    assert meta["blob_bytes"] <= sum(sts.values()) + 256 * (len(sts) + 4)  # + alignment + preprocess consts
    w_bytes = sum(pc.wf.numel() * 2 for pc in params.values() if hasattr(pc, "wf"))
    assert meta["blob_bytes"] >= w_bytes


def test_lite_runtime_imports_without_torch():
    code = ("import sys, hipzap.lite as L, hipzap.coldstart; "
            "assert 'torch' not in sys.modules, [m for m in sys.modules if m.startswith('torch')]; "
            "print(L.lib().hz_abi_version())")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert int(r.stdout.strip()) == N.lib().hz_abi_version()


def test_read_meta_and_abi_gate(tmp_path, r18):
    from hipzap import lite
    a, params, kw = r18
    path = str(tmp_path / "r18.hzplan")
    P.export_plan("resnet18", params, kw, path)
    meta = lite.read_meta(path)
    assert meta["model"] == "resnet18" and lite.plan_usable(path)
    raw = bytearray(open(path, "rb").read())
    raw[16:24] = (12345).to_bytes(8, "little")  # abi field
    bad = tmp_path / "bad.hzplan"
    bad.write_bytes(bytes(raw))
    assert not lite.plan_usable(str(bad))
    with pytest.raises(lite.PlanError):
        lite.read_meta(__file__)  # not a plan image


def test_sampled_digest_detects_same_size_replacement(tmp_path):
    from hipzap.engine.packfile import source_stamp
    p = tmp_path / "m.pth"
    p.write_bytes(os.urandom(3 << 20))
    st = os.stat(p)
    s1 = source_stamp(str(p))
    data = bytearray(p.read_bytes())
    data[0] ^= 0xFF  # the first sampled window always starts at byte 0
    p.write_bytes(bytes(data))
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))
    s2 = source_stamp(str(p))
    assert s1["size"] == s2["size"] and s1["mtime_ns"] == s2["mtime_ns"]
    assert s1["sampled_sha256"] != s2["sampled_sha256"]


def test_bert_text_plan_meta(tmp_path):
    """BERT exports as a TEXT plan: three adjacent host inputs (ids, token types,
    additive mask) that PlanTextBackend fills in one copy, and the table sizes the server checks
    request ids against."""
    from hipzap.lite import read_meta
    a = registry.get("bert-base")
    torch.manual_seed(0)
    from hipzap.models.bert import make_model
    m = make_model(2, num_hidden_layers=2)
    params, kw = a.pack(m.state_dict(), "cpu")
    path = str(tmp_path / "bert.hzplan")
    P.export_plan("bert-base", params, dict(kw), path, batch=4)
    meta = read_meta(path)
    assert meta["kind"] == "text" and meta["batch"] == 4 and meta["seq_len"] == 128
    assert meta["vocab"] == 30522 and meta["type_vocab"] == 2
    ins = meta["inputs"]
    assert [i["dtype"] for i in ins] == ["int32", "int32", "float32"]
    assert all(i["region"] == 2 for i in ins)
    assert all(ins[k]["off"] + ins[k]["bytes"] == ins[k + 1]["off"] for k in range(2)), ins
    assert meta["output"]["num_labels"] == 2


def _plan_open_error(path) -> str:
    """hz_plan_open on the CPU: parsing happens before the first HIP call, so a forged file is
    refused with a parse error; a well-formed one gets as far as device initialisation."""
    lib = N.lib()
    lib.hz_plan_open.restype = C.c_void_p
    lib.hz_plan_last_error.restype = C.c_char_p
    h = lib.hz_plan_open(str(path).encode(), 0, 1, None)
    if h:
        lib.hz_plan_close(C.c_void_p(h))
        return ""
    return lib.hz_plan_last_error().decode()


def test_plan_loader_refuses_forged_records(tmp_path, r18):
    import struct
    a, params, kw = r18
    path = tmp_path / "r18.hzplan"
    P.export_plan("resnet18", params, kw, str(path))
    raw = bytes(path.read_bytes())
    f = struct.unpack("<8s15Q", raw[:128])
    ops_off, ops_len = f[6], f[7]
    assert "truncated" not in _plan_open_error(path) and "shorter" not in _plan_open_error(path)

    def forged(name, data):
        p = tmp_path / name
        p.write_bytes(bytes(data))
        return _plan_open_error(p)

    # the first op's parameter record claims 8 bytes (its struct is far larger)
    b = bytearray(raw)
    typ, arg, slot, plen, nrel, pad = struct.unpack("<IiiIII", b[ops_off: ops_off + 24])
    b[ops_off + 12: ops_off + 16] = struct.pack("<I", 8)
    b[ops_off + 16: ops_off + 20] = struct.pack("<I", 0)
    assert "shorter than its parameters" in forged("short.hzplan", b) or "op record" in forged("short.hzplan", b)
    # a relocation offset that would wrap a 32-bit bound check
    b = bytearray(raw)
    if nrel:
        r0 = ops_off + 24 + ((plen + 7) & ~7)
        b[r0: r0 + 4] = struct.pack("<I", 0xFFFFFFFC)
        assert "relocation out of range" in forged("reloc.hzplan", b)
    # an ops table whose offset + length wraps around 2^64
    b = bytearray(raw)
    b[8 + 8 * 5: 8 + 8 * 6] = struct.pack("<Q", 2 ** 64 - 64)  # ops_off
    b[8 + 8 * 6: 8 + 8 * 7] = struct.pack("<Q", 128)           # ops_len
    assert "truncated file" in forged("wrap.hzplan", b)
    # an op whose record length runs past the table
    b = bytearray(raw)
    b[ops_off + 16: ops_off + 20] = struct.pack("<I", 0x7FFFFFFF)  # nrel
    assert "truncated op record" in forged("nrel.hzplan", b)
