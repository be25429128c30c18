"""Every global load / store address of the fp32 GEMM policies (qnet32_kernels.h) stays inside its buffer: the
launches qnet32.hip issues are replayed on the CPU (scripts/q32_host_check.hip, compiled host-only) against host
buffers of exactly the device workspace sizes under AddressSanitizer, with null frame-table entries (ring slots before
an episode's first frame) mixed in.  No GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("q32") / "q32_host_check")
    subprocess.run([HIPCC, "--offload-host-only", "-x", "hip", "-I", os.path.join(ROOT, "q-learning_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), "-fsanitize=address", "-g", "-O1",
                    os.path.join(ROOT, "scripts", "q32_host_check.hip"), "-o", exe], check=True, capture_output=True)
    return exe


@pytest.mark.parametrize("B,n", [(1, 1), (32, 128), (33, 200), (257, 257)])
def test_fp32_policy_addresses_in_bounds(checker, B, n):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    r = subprocess.run([checker, str(B), str(n)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "all in bounds" in r.stdout
