"""Host sanitizer builds (CPU): the bl::llama mirror, the request server and the wire format
(blama_amd/host) compiled with the C++ tests under ASan + UBSan and under TSan
(`make -C blama_amd/host san`), running the test binary's CPU cases: LogitComparer, the
sampler chain, the SPM tokenizer on a vocab-only model, the JSON wire format and its input
validation.  The GPU cases (sessions, server worker threads) need the device and run in the
plain build (tests/test_host.py)."""
import os
import subprocess

import pytest

from test_host import vocab_gguf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "cpp", "build")


@pytest.fixture(scope="module")
def san_bins():
    subprocess.run(["make", "-C", os.path.join(ROOT, "blama_amd", "host"), "san"], check=True,
                   capture_output=True, timeout=600)
    return {k: os.path.join(BUILD, f"t_bl_llama_{k}") for k in ("asan", "tsan")}


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_cpu_cases_under_sanitizer(san_bins, kind, tmp_path):
    v = str(tmp_path / "vocab.gguf")
    vocab_gguf(v)
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",      # the HIP runtime's own allocations
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([san_bins[kind], "cpu", f"--vocab={v}"], capture_output=True, text=True, timeout=300,
                       env=env)
    print(r.stdout[-3000:], r.stderr[-3000:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr
