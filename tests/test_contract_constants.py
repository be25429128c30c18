"""The numeric contract's constants are the same on both sides: the conv weight-gradient chunk sizes of include/qlx.h
(QLX_F32_WGRAD_CHUNK_CONV*, the product's) and of the fp32 chain oracle (oracle/qnet32_ref.cpp kSC*), and the fc1
forward's chain count (qnet32_kernels.h kFc1Chains / oracle kFc1Chains).  Text-level check, no GPU."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*p):
    return open(os.path.join(ROOT, *p)).read()


def test_wgrad_chunk_sizes_match_oracle():
    h = _read("include", "qlx.h")
    prod = {int(m.group(1)): int(m.group(2)) for m in re.finditer(r"#define QLX_F32_WGRAD_CHUNK_CONV(\d) (\d+)", h)}
    o = re.search(r"constexpr int kSC1 = (\d+), kSC2 = (\d+), kSC3 = (\d+);", _read("oracle", "qnet32_ref.cpp"))
    assert o, "oracle chunk constants"
    assert prod == {1: int(o.group(1)), 2: int(o.group(2)), 3: int(o.group(3))}, (prod, o.groups())


def test_fc1_chain_count_matches_oracle():
    k = re.search(r"#define QLX_FC1_CHAINS (\d+)", _read("q-learning_amd", "csrc", "qnet32_kernels.h"))
    o = re.search(r"constexpr int kFc1Chains = (\d+);", _read("oracle", "qnet32_ref.cpp"))
    assert k and o and int(k.group(1)) == int(o.group(1)), (k and k.group(1), o and o.group(1))


def test_conv_fwd_chain_count_matches_oracle():
    k = re.search(r"#define QLX_CONV_FWD_CHAINS (\d+)", _read("q-learning_amd", "csrc", "qnet32_kernels.h"))
    o = re.search(r"constexpr int kConvFwdChains = (\d+);", _read("oracle", "qnet32_ref.cpp"))
    assert k and o and int(k.group(1)) == int(o.group(1)), (k and k.group(1), o and o.group(1))
