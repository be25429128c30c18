// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product (libqlx).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
//
// Counter-based RNG used by the CPU restatement.  The reference draws every random
// number from `rand::thread_rng()` (rand 0.8.5, ChaCha12, OS-seeded, unseedable:
// /root/reference/src/Cargo.lock:2941-2952).  A seeded restatement therefore has to
// define its own bit source; we use Philox4x32-10 (Salmon et al., SC'11) and keep
// rand 0.8.5's *derivation algorithms* (how a u32/u64 becomes an f32 range sample,
// an f64 in [0,1), a u8 in [0,n) and a usize in [0,len)) exactly, so that only the
// raw bit stream differs from the reference.  Parity of the bit stream itself is
// "unpinned" (the reference stream is unseedable); derivations are restated from the
// published rand 0.8.5 source (src/distributions/uniform.rs, float.rs).
//
// Stream layout (shared definition with the product, restated independently there):
//   key   = {seed lo32, seed hi32}
//   ctr   = {block index, c1, c2, purpose}
//   word j of a stream = output word (j & 3) of block (j >> 2);
//   next_u64 = next_u32 (lo) | next_u32 (hi) << 32   (rand BlockRng::next_u64 order).
#pragma once
#include <cstdint>
#include <cstring>

namespace orc {

enum Purpose : uint32_t {
  P_BALL = 1,      // ball launch angle: c1 = env id, c2 = reset count
  P_ACT = 2,       // epsilon-greedy draws: c1 = env id, c2 = vector-step index
  P_SAMPLE = 3,    // replay index sampling: c1 = update index, c2 = rank
  P_INIT = 4,      // GlorotUniform init: c1 = variable index, c2 = 0
  P_SYNTH = 5,     // synthetic data for isolated kernel tests
};

static inline void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct Stream {
  uint32_t key[2];
  uint32_t c1, c2, purpose;
  uint64_t word = 0;
  uint32_t buf[4];
  uint64_t buf_block = ~0ull;

  Stream(uint64_t seed, uint32_t c1_, uint32_t c2_, uint32_t purpose_, uint64_t start_word = 0)
      : c1(c1_), c2(c2_), purpose(purpose_), word(start_word) {
    key[0] = (uint32_t)seed;
    key[1] = (uint32_t)(seed >> 32);
  }
  uint32_t next_u32() {
    const uint64_t blk = word >> 2;
    if (blk != buf_block) {
      const uint32_t ctr[4] = {(uint32_t)blk, c1, c2, purpose};
      philox4x32_10(ctr, key, buf);
      buf_block = blk;
    }
    const uint32_t v = buf[word & 3];
    ++word;
    return v;
  }
  uint64_t next_u64() {
    const uint64_t lo = next_u32();
    const uint64_t hi = next_u32();
    return lo | (hi << 32);
  }
};

static inline float f32_from_bits(uint32_t b) { float f; std::memcpy(&f, &b, 4); return f; }
static inline uint32_t f32_bits(float f) { uint32_t b; std::memcpy(&b, &f, 4); return b; }
static inline double f64_from_bits(uint64_t b) { double f; std::memcpy(&f, &b, 8); return f; }

// rand 0.8.5 UniformFloat<f32>::sample_single(low, high) — `rng.gen_range(low..high)`.
static inline float gen_range_f32(Stream& s, float low, float high) {
  float scale = high - low;
  for (;;) {
    const uint32_t bits = (s.next_u32() >> 9) | 0x3F800000u;   // [1,2)
    const float value0_1 = f32_from_bits(bits) - 1.0f;
    const float res = value0_1 * scale + low;
    if (res < high) return res;
    scale = f32_from_bits(f32_bits(scale) - 1u);
  }
}

// rand 0.8.5 UniformFloat<f64>::sample_single(0.0, 1.0) — `rng.gen_range(0_f64..1_f64)`
// (self_driving_tf_q_learner.rs:153).
static inline double gen_range_f64_01(Stream& s) {
  double scale = 1.0;
  for (;;) {
    const uint64_t bits = (s.next_u64() >> 12) | 0x3FF0000000000000ull;
    const double value0_1 = f64_from_bits(bits) - 1.0;
    const double res = value0_1 * scale + 0.0;
    if (res < 1.0) return res;
    uint64_t sb; std::memcpy(&sb, &scale, 8); --sb; std::memcpy(&scale, &sb, 8);
  }
}

// rand 0.8.5 UniformInt<u8>::sample_single(0, n) (large type u32, modulus zone) —
// `rng.gen_range(0..ACTION_SPACE)` (self_driving_tf_q_learner.rs:156).
static inline uint8_t gen_range_u8(Stream& s, uint8_t n) {
  const uint32_t range = n;                     // (high-1) - low + 1
  const uint32_t ints_to_reject = (0xFFFFFFFFu - range + 1u) % range;
  const uint32_t zone = 0xFFFFFFFFu - ints_to_reject;
  for (;;) {
    const uint32_t v = s.next_u32();
    const uint64_t m = (uint64_t)v * range;
    const uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
    if (lo <= zone) return (uint8_t)hi;
  }
}

// rand 0.8.5 Uniform<usize>::from(0..len).sample(rng) (u64, modulus zone from new_inclusive).
struct UniformUsize {
  uint64_t range, zone;
  explicit UniformUsize(uint64_t len) : range(len) {
    const uint64_t ints_to_reject = range > 0 ? (UINT64_MAX - range + 1) % range : 0;
    zone = UINT64_MAX - ints_to_reject;
  }
  uint64_t sample(Stream& s) const {
    for (;;) {
      const uint64_t v = s.next_u64();
      const unsigned __int128 m = (unsigned __int128)v * range;
      const uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
      if (lo <= zone) return hi;
    }
  }
};

}  // namespace orc
