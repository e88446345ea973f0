"""Host AddressSanitizer + UBSan run of the native runtime (SURVEY.md §5 'race detection /
sanitizers'): csrc/runtime.cpp is compiled with ``-Xarch_host -fsanitize=address,undefined``
(host code only — GPU ASan is not used) together with tests/native/runtime_host_asan.cpp, whose
stub kernel launchers let the Program container run without a GPU. Leak detection is on."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_runtime_host_asan_ubsan(tmp_path):
    exe = tmp_path / "rt_asan"
    san = []
    for f in ("-fsanitize=address", "-fsanitize=undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"):
        san += ["-Xarch_host", f]
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", *san, "-I", os.path.join(ROOT, "hipzap", "csrc"),
           os.path.join(ROOT, "hipzap", "csrc", "runtime.cpp"),
           os.path.join(ROOT, "tests", "native", "runtime_host_asan.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0 and "runtime host asan: ok" in run.stdout, (run.stdout[-2000:], run.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in run.stderr and "runtime error" not in run.stderr


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("sanitizer", ["address,undefined", "thread"])
def test_http_parsers_fuzz_asan_ubsan(tmp_path, sanitizer):
    """The native HTTP front end's body parsers (JSON image, .npy, base64, int arrays) on 200k
    mutated / random inputs held in exact-size heap blocks, its request framing (serve_conn
    over a socketpair: pipelined, truncated, chunked, negative lengths), and the whole server over
    loopback TCP with hz_http_stop racing connecting clients -- under host ASan + UBSan and
    under ThreadSanitizer."""
    exe = tmp_path / f"http_fuzz_{sanitizer.split(',')[0]}"
    san = []
    for f in (f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"):
        san += ["-Xarch_host", f]
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", *san, "-I", os.path.join(ROOT, "hipzap", "csrc"),
           os.path.join(ROOT, "tests", "native", "http_parse_fuzz.cpp"), "-lpthread", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0 and "http parse fuzz: ok" in run.stdout, (run.stdout[-2000:], run.stderr[-4000:])
    for marker in ("ERROR: AddressSanitizer", "runtime error", "WARNING: ThreadSanitizer"):
        assert marker not in run.stderr, run.stderr[-4000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("sanitizer", ["address,undefined", "thread"])
def test_executor_host_sanitizers(tmp_path, sanitizer):
    """The request executor (csrc/executor.cpp) under host ASan+UBSan and under ThreadSanitizer:
    concurrent single-row, dynamic-batching and multi-row (hz_exec_submit_rows) requests against a
    fake program that computes each row at replay time, so a launch before the rows are copied or a
    read before the replay is a wrong answer, and any unsynchronised slot access is a TSan report."""
    exe = tmp_path / f"exec_{sanitizer.split(',')[0]}"
    san = []
    for f in (f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"):
        san += ["-Xarch_host", f]
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", *san, "-I", os.path.join(ROOT, "hipzap", "csrc"),
           os.path.join(ROOT, "hipzap", "csrc", "executor.cpp"),
           os.path.join(ROOT, "tests", "native", "executor_host_sanitize.cpp"), "-lpthread", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0 and "executor host sanitize: ok" in run.stdout, (run.stdout[-2000:], run.stderr[-4000:])
    for marker in ("ERROR: AddressSanitizer", "runtime error", "WARNING: ThreadSanitizer"):
        assert marker not in run.stderr, run.stderr[-4000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("sanitizer", ["address,undefined", "thread"])
def test_lmserve_host_sanitizers(tmp_path, sanitizer):
    """The batched-decode scheduler (csrc/lmserve.cpp): pipelined program pair, alternating output
    slots, low-load switch, logits recording, under host ASan+UBSan and ThreadSanitizer against an
    in-order fake device that reads each host block only when its replay runs."""
    exe = tmp_path / f"lmserve_{sanitizer.split(',')[0]}"
    san = []
    for f in (f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"):
        san += ["-Xarch_host", f]
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", *san, "-I", os.path.join(ROOT, "hipzap", "csrc"),
           os.path.join(ROOT, "hipzap", "csrc", "lmserve.cpp"),
           os.path.join(ROOT, "tests", "native", "lmserve_host_sanitize.cpp"), "-lpthread", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0 and "lmserve host sanitize: ok" in run.stdout, (run.stdout[-2000:], run.stderr[-4000:])
    for marker in ("ERROR: AddressSanitizer", "runtime error", "WARNING: ThreadSanitizer"):
        assert marker not in run.stderr, run.stderr[-4000:]
