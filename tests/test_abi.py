"""The C ABI boundary without a GPU: libqlx.so loads, exports every entry point include/qlx.h declares, answers
the pure host queries, and fails loudly (QlError, no CPU fallback) when a call needs a device that is absent.
The product library links no part of oracle/."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "qlx.h")
LIB = os.path.join(ROOT, "q-learning_amd", "lib", "libqlx.so")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(qlx_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    assert os.path.exists(LIB), "libqlx.so not built (make lib)"
    return ctypes.CDLL(LIB)


def test_header_declares_the_reference_surface():
    names = set(_declared())
    # the trait surface of SURVEY.md §8(b): env, replay, model, learner, data parallel
    for n in ["qlx_env_create", "qlx_env_step", "qlx_env_reset", "qlx_env_obs", "qlx_replay_create", "qlx_replay_push",
              "qlx_replay_sample_distinct", "qlx_model_create", "qlx_model_predict", "qlx_model_batch_max_q",
              "qlx_model_train", "qlx_model_write_checkpoint", "qlx_learner_create", "qlx_learner_run",
              "qlx_learner_dist_init", "qlx_last_error"]:
        assert n in names, n


def test_every_declared_entry_point_is_exported(lib):
    names = _declared()
    assert len(names) > 90
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and as dynamic symbols of the shared object (what cgo / a Rust extern block would bind)
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    dyn = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not [n for n in names if n not in dyn]


def test_host_queries_without_device(lib):
    lib.qlx_version.restype = ctypes.c_int32
    lib.qlx_env_action_space.restype = ctypes.c_int32
    lib.qlx_env_reward_goal_mean.restype = ctypes.c_float
    assert lib.qlx_version() >= 1
    # breakout_environment.rs:104-119 (3 actions), ballgame_test_environment.rs (5); goal means :203-206 / 9.5
    breakout, ballgame = 1, 2   # QLX_ENV_BREAKOUT / QLX_ENV_BALLGAME
    assert lib.qlx_env_action_space(breakout) == 3
    assert lib.qlx_env_action_space(ballgame) == 5
    assert lib.qlx_env_action_space(7) == -1
    assert lib.qlx_env_reward_goal_mean(breakout) == 59.0
    assert lib.qlx_env_reward_goal_mean(ballgame) == 9.5


def test_device_calls_fail_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the device path is covered by the -m gpu tests")
    import qlx
    with pytest.raises(qlx.QlError, match="device"):
        qlx.BreakoutEnvironment(4)
    with pytest.raises(qlx.QlError):
        qlx.SelfDrivingQLearner(qlx.Parameter(n_envs=16, batch_size=32, history_buffer_len=1000))


def test_product_links_no_oracle():
    out = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"\(NEEDED\).*\[(.*)\]", out)
    assert needed and not [n for n in needed if "oracle" in n], needed
    syms = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True, check=True).stdout
    assert "oracle" not in syms.lower()
