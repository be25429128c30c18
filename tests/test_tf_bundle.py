"""TF tensor-bundle reader (q-learning_amd/csrc/tf_bundle.cpp, host code: runs without a GPU) on the reference's
own SavedModel variables (tests/golden/, see its README): every name / dtype / shape the Keras models declare
(create_ql_model_*.py), block and tensor crc32c verified, and the values the reference's export holds
(GlorotUniform kernels within +-sqrt(6 / (fan_in + fan_out)), zero biases, zero Adam slots, iter 0)."""
import os

import numpy as np
import pytest

import qlx

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BG = os.path.join(GOLD, "ballgame_saved_variables", "variables")
BO = os.path.join(GOLD, "breakout_saved_variables", "variables")


def var_name(layer, kind, slot=None):
    base = f"layer_with_weights-{layer}/{kind}"
    if slot is None:
        return base + "/.ATTRIBUTES/VARIABLE_VALUE"
    return base + f"/.OPTIMIZER_SLOT/optimizer/{slot}/.ATTRIBUTES/VARIABLE_VALUE"


def test_ballgame_bundle_names_shapes_values():
    b = qlx.TfBundle(BG)
    ents = b.entries()
    fans = [(2 * 2 * 4, 2 * 2 * 32), (32, 32), (288, 512), (512, 5)]
    for v, shape in enumerate(qlx.BG_VAR_SHAPES):
        layer, kind = v // 2, ("kernel", "bias")[v % 2]
        for slot in (None, "m", "v"):
            dt, sh, nb = ents[var_name(layer, kind, slot)]
            assert dt == 1 and sh == shape and nb == 4 * int(np.prod(shape))
        w = b.read(var_name(layer, kind))
        if kind == "kernel":
            lim = np.sqrt(6.0 / sum(fans[layer]))
            assert np.abs(w).max() <= lim and np.abs(w).max() > 0.9 * lim   # GlorotUniform
            assert abs(float(w.mean())) < 0.1 * lim
        else:
            assert not w.any()
        assert not b.read(var_name(layer, kind, "m")).any() and not b.read(var_name(layer, kind, "v")).any()
    assert int(b.read("optimizer/iter/.ATTRIBUTES/VARIABLE_VALUE")) == 0
    assert np.isclose(float(b.read("optimizer/learning_rate/.ATTRIBUTES/VARIABLE_VALUE")), 0.00025)
    assert np.isclose(float(b.read("optimizer/beta_1/.ATTRIBUTES/VARIABLE_VALUE")), 0.9)
    assert np.isclose(float(b.read("optimizer/beta_2/.ATTRIBUTES/VARIABLE_VALUE")), 0.999)


def test_breakout_index_matches_the_nature_dqn_layout():
    b = qlx.TfBundle(BO)
    ents = b.entries()
    for v, shape in enumerate(qlx.VAR_SHAPES):
        dt, sh, nb = ents[var_name(v // 2, ("kernel", "bias")[v % 2])]
        assert dt == 1 and sh == tuple(shape) and nb == 4 * int(np.prod(shape))
    with pytest.raises(qlx.QlError):   # the data blob is not part of the reference checkout
        b.read(var_name(0, "kernel"))


def test_corrupt_bundle_is_rejected(tmp_path):
    raw = bytearray(open(BG + ".index", "rb").read())
    raw[100] ^= 0xFF                                   # inside a data block: block crc32c mismatch
    (tmp_path / "variables.index").write_bytes(bytes(raw))
    with pytest.raises(qlx.QlError):
        qlx.TfBundle(str(tmp_path / "variables"))
