"""The oracle's reference-loop restatement (breakout physics + raster, replay, sampler, learner loop, fp32 Q-net train
step) built host-only under AddressSanitizer + UndefinedBehaviorSanitizer and run for a short loop: no invalid access,
leak or undefined behaviour in the checker itself (SURVEY §5 auxiliaries: host sanitizer build of the oracle)."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_oracle_loop_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "cpu_baseline_asan")
    srcs = ["cpu_baseline.cpp", "breakout_ref.cpp", "qnet_ref.cpp", "learner_ref.cpp", "qnet32_ref.cpp"]
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-mfma",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer",
                    "-o", exe] + [os.path.join(ORACLE, s) for s in srcs], check=True, capture_output=True)
    env = dict(os.environ, OMP_NUM_THREADS="4", ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    # 120 env-steps, one env, B = 8: the pure-random phase with updates from step 9 on (~28 fp32 train steps)
    r = subprocess.run([exe, "120", "1", "8"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["env_steps"] == 120 and out["updates"] > 20
