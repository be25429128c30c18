// Batched Breakout environment on MI355X (gfx950): one lane per env for the physics tick, one wave
// per env for the 84x84 frame (space-to-depth layout, 16-byte stores).
//
// Reference behaviour (restated, not ported):
//   BreakoutMechanics::time_step        src/breakout-game/src/mechanics.rs:119-135
//   Panel::proceed / process_input      mechanics.rs:553-588;  decrease/accelerate/granulate :612-649
//   proceed_ball_with (recursive)        mechanics.rs:137-184 -> bounded loop below
//   check_collisions / ContactCandidates mechanics.rs:186-213, 485-539 -> two-pass candidate scan
//   wall tests / rectangle contact       mechanics.rs:260-443, algebra_2d.rs:47-75 (+ parry2d contact)
//   BreakoutEnvironment::step / reset    src/_breakout-ml/src/breakout_environment.rs:173-201
//   FrameRingBuffer::add                 src/_breakout-ml/src/util/frame_ring_buffer.rs:53-63
// This translation unit is compiled with -ffp-contract=off: every a*b+c rounds twice, as in Rust.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "objects.h"

namespace qlx {

namespace phys {

constexpr float kGrid = 600.0f;
constexpr float kSpaceGranularity = 0.001f;
constexpr float kPrediction = 0.8f;
constexpr float kFracPi2 = 1.57079637050628662109375f;
constexpr int kMaxMoves = 64;
constexpr int kMaxBisect = 64;

struct F2 { float x, y; };
__device__ __forceinline__ F2 add(F2 a, F2 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ F2 sub(F2 a, F2 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ F2 scale(F2 a, float s) { return {a.x * s, a.y * s}; }
__device__ __forceinline__ F2 divs(F2 a, float s) { return {a.x / s, a.y / s}; }
__device__ __forceinline__ float dotp(F2 a, F2 b) { return a.x * b.x + a.y * b.y; }
// emath Vec2::length = f32::hypot -> glibc: (float) sqrt((double)x*x + (double)y*y)
__device__ __forceinline__ float length(F2 a) {
  const double x = a.x, y = a.y;
  return (float)__builtin_sqrt(x * x + y * y);
}
__device__ __forceinline__ F2 normalized(F2 a) {
  const float l = length(a);
  return l <= 0.0f ? a : divs(a, l);
}

struct Surface { float way, approx; F2 n; };

// parry2d contact(ball, cuboid) -> (dist, ball-side normal, cuboid outward normal)
__device__ bool contact(F2 c, float r, float x0, float y0, float x1, float y1, float* dist, F2* n_ball, F2* n_box) {
  const F2 bc = {(x0 + x1) / 2.0f, (y0 + y1) / 2.0f};
  const F2 he = {(x1 - x0) / 2.0f, (y1 - y0) / 2.0f};
  const F2 p = {-(bc.x - c.x), -(bc.y - c.y)};        // ball centre in the cuboid frame
  const float mins_x = -he.x - p.x, mins_y = -he.y - p.y;
  const float maxs_x = p.x - he.x, maxs_y = p.y - he.y;
  const float sx = fmaxf(mins_x, 0.0f) - fmaxf(maxs_x, 0.0f);
  const float sy = fmaxf(mins_y, 0.0f) - fmaxf(maxs_y, 0.0f);
  const bool inside = sx == 0.0f && sy == 0.0f;
  F2 proj;
  if (!inside) {
    proj = {p.x + sx, p.y + sy};
  } else {
    // nearest face: the largest of the (non-positive) face distances, first axis wins ties
    float best = -FLT_MAX, shx = 0.0f, shy = 0.0f;
    int id = 0;
    if (mins_x < maxs_x) { if (maxs_x > best) { best = maxs_x; id = 1; } } else if (mins_x > best) { best = mins_x; id = -1; }
    if (mins_y < maxs_y) { if (maxs_y > best) { best = maxs_y; id = 2; } } else if (mins_y > best) { best = mins_y; id = -2; }
    if (id == 1) shx = -best; else if (id == -1) shx = best; else if (id == 2) shy = -best; else shy = best;
    proj = {p.x + shx, p.y + shy};
  }
  const F2 d = sub(proj, p);
  const float sq = d.x * d.x + d.y * d.y;
  float dd;
  F2 n1;
  if (sq > FLT_EPSILON * FLT_EPSILON) {
    const float len = __builtin_sqrtf(sq);
    const F2 dir = divs(d, len);
    if (inside) { dd = -len - r; n1 = dir; } else { dd = len - r; n1 = {-dir.x, -dir.y}; }
  } else {
    // centre exactly on the boundary: face normal, vertex (diagonal) normal on a corner
    dd = -r;
    const float fx = p.x >= he.x - FLT_EPSILON ? 1.0f : (p.x <= -he.x + FLT_EPSILON ? -1.0f : 0.0f);
    const float fy = p.y >= he.y - FLT_EPSILON ? 1.0f : (p.y <= -he.y + FLT_EPSILON ? -1.0f : 0.0f);
    if (fx != 0.0f && fy != 0.0f) n1 = divs(F2{fx, fy}, __builtin_sqrtf(fx * fx + fy * fy));
    else if (fx != 0.0f || fy != 0.0f) n1 = {fx, fy};
    else n1 = {0.0f, 1.0f};
  }
  if (dd <= kPrediction) {
    *dist = dd;
    *n_ball = {-n1.x, -n1.y};
    *n_box = n1;
    return true;
  }
  return false;
}

// Ball::collision_check_with_rectangle + find_non_penetrating_collision (mechanics.rs:318-443)
__device__ bool rect_surface(F2 c, float r, F2 mv, float x0, float y0, float x1, float y1, float acos_thr,
                             Surface* out, uint32_t* fault) {
  float dist;
  F2 nb, nx;
  if (!contact(add(c, mv), r, x0, y0, x1, y1, &dist, &nb, &nx)) return false;
  Surface s;
  if (dist < -0.0f) {
    const float mvlen = length(mv);
    const float x = fabsf(dist) / (dotp(nb, mv) / mvlen);
    const float portion = 1.0f - x / mvlen;
    float d2;
    F2 nb2, nx2;
    const bool hit2 = contact(add(c, scale(mv, portion)), r, x0, y0, x1, y1, &d2, &nb2, &nx2);
    if (hit2 && !(d2 < -0.0f)) {
      s = {mvlen * portion, d2, nx2};
    } else {
      float lo = hit2 ? 0.0f : portion, hi = hit2 ? portion : 1.0f;
      bool found = false;
      for (int it = 0; it <= kMaxBisect; ++it) {
        const float m = (lo + hi) / 2.0f;
        float d3;
        F2 nb3, nx3;
        if (!contact(add(c, scale(mv, m)), r, x0, y0, x1, y1, &d3, &nb3, &nx3)) lo = m;
        else if (d3 < -0.0f) hi = m;
        else { s = {mvlen * m, d3, nx3}; found = true; break; }
      }
      if (!found) { *fault |= 4u; s = {mvlen * hi, 0.0f, F2{0.0f, 1.0f}}; }
    }
  } else {
    s = {length(mv), dist, nx};
  }
  // accept only contacts within +-90 deg of the move: acos(n(mv) . n(normal)) > FRAC_PI_2
  // <=> dot < acos_thr (threshold precomputed from libm acosf on the host, exact equivalence).
  const float d = dotp(normalized(mv), normalized(s.n));
  if (!(d < acos_thr)) return false;
  *out = s;
  return true;
}

struct Ctx {
  F2 c;
  float r;
  F2 mv;
  float panel[4];
  uint64_t bricks;
  float acos_thr;
};

__device__ __forceinline__ void brick_box(int id, float* b) {
  const int row = id / 20, col = id - row * 20;
  b[0] = 30.0f + 27.0f * (float)col;
  b[2] = b[0] + 25.0f;
  b[3] = 60.0f + 27.0f * (float)row;
  b[1] = b[3] - 25.0f;
}

// candidate object o: 0 left wall, 1 right wall, 2 top wall, 3 panel, 4 + id bricks (creation order)
__device__ bool candidate(const Ctx& x, int o, Surface* s, uint32_t* fault) {
  if (o == 0) {
    const float w = x.c.x - x.r;
    if (!(w >= 0.0f)) *fault |= 1u;
    if (w + x.mv.x > 0.0f) return false;
    *s = {length(scale(x.mv, w / fabsf(x.mv.x))), 0.0f, F2{1.0f, 0.0f}};
    return true;
  }
  if (o == 1) {
    const float w = kGrid - x.c.x - x.r;
    if (!(w >= 0.0f)) *fault |= 1u;
    if (x.mv.x < w) return false;
    *s = {length(scale(x.mv, w / fabsf(x.mv.x))), 0.0f, F2{-1.0f, 0.0f}};
    return true;
  }
  if (o == 2) {
    const float w = x.c.y - x.r - 0.0f;
    if (!(w >= 0.0f)) *fault |= 1u;
    if (w + x.mv.y > 0.0f) return false;
    *s = {length(scale(x.mv, w / fabsf(x.mv.y))), 0.0f, F2{0.0f, 1.0f}};
    return true;
  }
  float b[4];
  if (o == 3) { b[0] = x.panel[0]; b[1] = x.panel[1]; b[2] = x.panel[2]; b[3] = x.panel[3]; }
  else brick_box(o - 4, b);
  // conservative early-out: a contact needs the end position within r + 0.8 of the box
  const float ex = x.c.x + x.mv.x, ey = x.c.y + x.mv.y;
  const float reach = x.r + kPrediction + 1.0f;
  if (ex < b[0] - reach || ex > b[2] + reach || ey < b[1] - reach || ey > b[3] + reach) return false;
  return rect_surface(x.c, x.r, x.mv, b[0], b[1], b[2], b[3], x.acos_thr, s, fault);
}

__device__ __forceinline__ float granulate(float s) { return roundf(s * 1000.0f) / 1000.0f; }

}  // namespace phys

// Per-env state (public ABI struct), 64 bytes.
using State = qlx_breakout_state;

__device__ void init_state(State& s, uint64_t seed, uint32_t env, uint32_t reset_count) {
  RngStream rs(seed, env, reset_count, P_BALL);
  s.ball_x = 600.0f * 0.5f;
  s.ball_y = 600.0f * 0.5f;
  s.dir_x = uniform_f32(rs, -0.35f, -0.15f);
  s.dir_y = -1.0f;
  s.panel_min_x = 600.0f / 2.0f - 60.0f / 2.0f;
  s.panel_min_y = (600.0f - 30.0f) - 10.0f / 2.0f;
  s.panel_max_x = 600.0f / 2.0f + 60.0f / 2.0f;
  s.panel_max_y = (600.0f - 30.0f) + 10.0f / 2.0f;
  s.panel_speed = 0.0f;
  s.score = 0;
  s.finished = 0;
  s.next_slot = 0;
  s.fault = 0;
  s.reset_count = reset_count;
  s.bricks = (1ull << kNumBricks) - 1ull;
}

// One physics tick (BreakoutMechanics::time_step) for one env, computed by one wave: every lane holds the same
// ball / panel state, lane o tests contact object o (4 + 60 objects = 64 lanes), and the candidate sums are
// taken lane by lane in object order, so every float operation is the sequential one.
static_assert(4 + kNumBricks <= 64, "one lane per contact object");
__device__ void time_step(State& s, uint32_t action, float acos_thr, int lane) {
  using namespace phys;
  const float tg = 20000000.0f / 1000000000.0f;   // TIME_GRANULARITY.as_secs_f32()
  // Panel::proceed
  {
    const float dx = s.panel_speed * tg;
    const float mnx = s.panel_min_x + dx, mxx = s.panel_max_x + dx;
    if (mnx <= 0.0f) {
      const float t = -mnx;
      s.panel_min_x = mnx + t; s.panel_max_x = mxx + t; s.panel_speed = 0.0f;
    } else if (mxx >= kGrid) {
      const float t = kGrid - mxx;
      s.panel_min_x = mnx + t; s.panel_max_x = mxx + t; s.panel_speed = 0.0f;
    } else {
      s.panel_min_x = mnx; s.panel_max_x = mxx;
    }
  }
  // proceed_ball_with(move_vector)
  Ctx x;
  x.c = {s.ball_x, s.ball_y};
  x.r = 10.0f;
  F2 dir = {s.dir_x, s.dir_y};
  x.mv = scale(scale(normalized(dir), 200.0f), tg);
  x.panel[0] = s.panel_min_x; x.panel[1] = s.panel_min_y; x.panel[2] = s.panel_max_x; x.panel[3] = s.panel_max_y;
  x.bricks = s.bricks;
  x.acos_thr = acos_thr;
  uint32_t fault = 0;   // this lane's fault bits (OR-reduced below)
  const int o = lane;      // the object this lane tests: 0-3 walls / panel, 4 + id bricks (creation order)
  for (int move = 0;; ++move) {
    if (length(x.mv) < kSpaceGranularity) break;
    if (move > kMaxMoves) { fault |= 4u; break; }
    // pass 1, one object per lane: candidate, count, shortest path (ContactCandidates::consider asserts the
    // approximation range of every inserted candidate).  The sequential "if (pl < shortest)" keeps the
    // least non-NaN path, which a min reduction gives in any order.
    const bool alive = o < 4 || ((x.bricks >> (o - 4)) & 1ull);
    Surface su = {0.0f, 0.0f, F2{0.0f, 0.0f}};
    const bool hit = alive && candidate(x, o, &su, &fault);
    if (hit && !(su.approx >= -0.0f && su.approx <= kPrediction)) fault |= 2u;
    const float pl = su.way + su.approx;
    float shortest = hit && pl == pl ? pl : INFINITY;
    for (int off = 32; off > 0; off >>= 1) shortest = fminf(shortest, __shfl_xor(shortest, off));
    const uint64_t hitmask = __ballot(hit);
    const int count = __builtin_popcountll(hitmask);
    if (count == 0) { x.c = add(x.c, x.mv); break; }
    // pass 2: ContactCandidates::consider keeps {path <= shortest + 0.001} (any single candidate if it is the
    // only one); sums run in insertion order (walls, panel, bricks ascending) = lane order, read lane by lane
    const float thr = shortest + kSpaceGranularity;
    F2 nsum = {0.0f, 0.0f};
    float asum = 0.0f, wsum = 0.0f;
    int kept = 0;
    Surface first = {0.0f, 0.0f, F2{0.0f, 0.0f}};
    uint64_t removed = 0;
    auto rl = [](float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); };
    for (uint64_t m = hitmask; m; m &= m - 1) {
      const int oh = __builtin_ctzll(m);
      const Surface c = {rl(su.way, oh), rl(su.approx, oh), F2{rl(su.n.x, oh), rl(su.n.y, oh)}};
      if (count > 1 && !(c.way + c.approx <= thr)) continue;
      if (kept == 0) first = c;
      nsum = add(nsum, c.n);
      asum = asum + c.approx;
      wsum = wsum + c.way;
      ++kept;
      if (oh >= 4) removed |= 1ull << (oh - 4);
    }
    const int nrem = __builtin_popcountll(removed);
    x.bricks &= ~removed;
    s.score += (uint32_t)nrem;
    if (kept == 0) { x.c = add(x.c, x.mv); break; }
    Surface col;
    if (kept == 1) col = first;
    else col = {wsum / (float)kept, asum / (float)kept, normalized(nsum)};
    const F2 cpos = add(x.c, scale(dir, col.way));
    const float remaining = length(x.mv) - col.way;
    const F2 refl = normalized(sub(dir, scale(col.n, 2.0f * dotp(dir, col.n))));
    x.c = cpos;
    dir = refl;
    const F2 rem = scale(refl, remaining);
    if (length(rem) > 0.0f) { x.mv = rem; continue; }
    break;
  }
  for (int off = 32; off > 0; off >>= 1) fault |= (uint32_t)__shfl_xor((int)fault, off);
  s.ball_x = x.c.x; s.ball_y = x.c.y;
  s.dir_x = dir.x; s.dir_y = dir.y;
  s.bricks = x.bricks;
  s.fault |= fault;
  // check_game_end_situation
  if (s.ball_y >= s.panel_max_y || s.bricks == 0) s.finished = 1;
  if (!s.finished) {
    const float v = s.panel_speed;
    if (action == 0) {
      s.panel_speed = v > 0.0f ? fmaxf(phys::granulate(v - 7.0f), 0.0f)
                               : (v < 0.0f ? fmaxf(phys::granulate(v + 7.0f), 0.0f) : 0.0f);
    } else {
      const float a = action == 1 ? -20.0f : 20.0f;
      const float vv = v + a;
      const float res = fabsf(vv) > 160.0f ? (signbit(vv) ? -160.0f : 160.0f) : vv;
      s.panel_speed = phys::granulate(res);
    }
  }
}

// ---------------------------------------------------------------------------------------
// kernels

// Reset of the envs selected by mask (all if null), one block per env: new state (init_state) and the 4 ring
// frames zeroed (FrameRingBuffer::new).  Unselected envs return at once.
__global__ __launch_bounds__(256) void k_env_reset(State* st, uint32_t* ep_steps, uint8_t* obs, uint32_t n, uint64_t seed,
                                                   uint32_t id_offset, const uint8_t* mask, int bump) {
  const uint32_t e = blockIdx.x;
  if (e >= n || (mask && !mask[e])) return;
  if (threadIdx.x == 0) {
    const uint32_t rc = bump ? st[e].reset_count + 1 : 0;
    State s;
    init_state(s, seed, id_offset + e, rc);
    st[e] = s;
    ep_steps[e] = 0;
  }
  uint4* dst = reinterpret_cast<uint4*>(obs + (size_t)e * kSlots * kFramePix);
  const uint4 z = {0, 0, 0, 0};
  for (uint32_t i = threadIdx.x; i < kSlots * kFramePix / 16; i += 256) dst[i] = z;
}

// one wave per env (4 envs per 256-thread block)
__global__ __launch_bounds__(256) void k_env_step(State* st, uint32_t* ep_steps, uint32_t n, const uint8_t* actions, float* rewards,
                                                  uint8_t* dones, float acos_thr, uint32_t* bad_action) {
  const uint32_t e = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= n) return;
  State s = st[e];
  uint32_t a = actions[e];
  if (a >= kActions) {
    if (lane == 0) atomicOr(bad_action, 1u);
    a = 0;
  }
  const uint32_t prev = s.score;
  time_step(s, a, acos_thr, lane);
  s.next_slot = (s.next_slot + 1) & 3;   // FrameRingBuffer::add advances; the frame goes to the old slot
  if (lane == 0) {
    st[e] = s;
    rewards[e] = (float)(s.score - prev);
    dones[e] = (uint8_t)s.finished;
    ep_steps[e] += 1;
  }
}

__constant__ int8_t c_brick_col[kFrame];
__constant__ int8_t c_brick_row[kFrame];

__device__ __forceinline__ uint64_t fbits_h(float f) { return f == 0.0f ? 0ull : (uint64_t)f32_bits(f); }

// One 256-thread block per env: rasterise the frame of the step just taken into ring slot (next_slot - 1) & 3,
// s2d layout (441 16-pixel blocks, ~2 per thread); HASH folds it into the env's running checksum (wrapping u64
// sums: any reduction order gives the same bits).
template <bool HASH>
__global__ __launch_bounds__(256) void k_env_raster(const State* st, uint32_t n, uint8_t* obs, uint64_t* hashes) {
  const uint32_t e = blockIdx.x;
  const int tid = threadIdx.x;
  if (e >= n) return;
  const State s = st[e];
  const int slot = (s.next_slot + 3) & 3;
  uint8_t* frame = obs + ((size_t)e * kSlots + slot) * kFramePix;
  const float S = 600.0f / 84.0f;
  const float rr = 10.0f * 10.0f;
  uint64_t hf = 0;
  for (int blk = tid; blk < kBlocks * kBlocks; blk += 256) {
    const int X = blk / kBlocks, Y = blk - X * kBlocks;   // X: image x / 4, Y: image y / 4
    uint32_t w[4];
#pragma unroll
    for (int dx = 0; dx < 4; ++dx) {
      const int px = 4 * X + dx;
      const float wx = ((float)px + 0.5f) * S;
      const int bc = c_brick_col[px];
      uint32_t word = 0;
#pragma unroll
      for (int dy = 0; dy < 4; ++dy) {
        const int py = 4 * Y + dy;
        const float wy = ((float)py + 0.5f) * S;
        uint32_t v = 0;
        const int br = c_brick_row[py];
        if (bc >= 0 && br >= 0 && ((s.bricks >> (br * 20 + bc)) & 1ull)) v = 96;
        if (s.panel_min_x <= wx && wx < s.panel_max_x && s.panel_min_y <= wy && wy < s.panel_max_y) v = 255;
        const float ddx = wx - s.ball_x, ddy = wy - s.ball_y;
        if (ddx * ddx + ddy * ddy <= rr) v = 236;
        word |= v << (8 * dy);
        if constexpr (HASH) hf += (uint64_t)v * ((uint64_t)(py * kFrame + px + 1) * kH1);
      }
      w[dx] = word;
    }
    reinterpret_cast<uint4*>(frame)[blk] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  if constexpr (HASH) {
    __shared__ uint64_t part[4];
    for (int off = 32; off > 0; off >>= 1) hf += __shfl_xor(hf, off);
    if ((tid & 63) == 0) part[tid >> 6] = hf;
    __syncthreads();
    if (tid == 0) {
      hf = part[0] + part[1] + part[2] + part[3];
      const uint64_t f[15] = {fbits_h(s.ball_x), fbits_h(s.ball_y), fbits_h(s.dir_x), fbits_h(s.dir_y),
                              fbits_h(s.panel_min_x), fbits_h(s.panel_min_y), fbits_h(s.panel_max_x),
                              fbits_h(s.panel_max_y), fbits_h(s.panel_speed), s.score, s.finished, s.next_slot,
                              s.fault, s.reset_count, s.bricks};
      uint64_t hs = 0;
      for (int j = 0; j < 15; ++j) hs += f[j] * ((uint64_t)(j + 1) * kH2);
      hashes[e] = hashes[e] * kH3 + hf + hs;
    }
  }
}

// obs (s2d ring) -> reference tensor view [n][x][y][slot]
__global__ void k_env_obs_view(const uint8_t* obs, uint32_t n, uint8_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // over n * 84 * 84
  if (i >= (size_t)n * kFramePix) return;
  const uint32_t e = (uint32_t)(i / kFramePix);
  const int xy = (int)(i - (size_t)e * kFramePix);
  const int x = xy / kFrame, y = xy - x * kFrame;
  const int off = s2d_offset(x, y);
  uchar4 v;
  v.x = obs[((size_t)e * kSlots + 0) * kFramePix + off];
  v.y = obs[((size_t)e * kSlots + 1) * kFramePix + off];
  v.z = obs[((size_t)e * kSlots + 2) * kFramePix + off];
  v.w = obs[((size_t)e * kSlots + 3) * kFramePix + off];
  reinterpret_cast<uchar4*>(out)[i] = v;
}

// ---------------------------------------------------------------------------------------
// host object

float acos_threshold_host() {
  // acosf(d) > FRAC_PI_2  <=>  d < T for the libm acosf the reference calls (f32::acos).
  float d = -1e-5f;
  while (std::acos(d) > phys::kFracPi2) d = std::nextafter(d, 1.0f);
  return d;
}

static void brick_luts(int8_t* col, int8_t* row) {
  const float S = 600.0f / 84.0f;
  for (int p = 0; p < kFrame; ++p) {
    const float w = ((float)p + 0.5f) * S;
    col[p] = -1;
    row[p] = -1;
    for (int k = 0; k < 20; ++k)
      if (30.0f + 27.0f * (float)k <= w && w < 30.0f + 27.0f * (float)k + 25.0f) col[p] = (int8_t)k;
    for (int r = 0; r < 3; ++r)
      if (35.0f + 27.0f * (float)r <= w && w < 60.0f + 27.0f * (float)r) row[p] = (int8_t)r;
  }
}

}  // namespace qlx

namespace qlx {

void env_launch_step(qlx_env* env, const uint8_t* d_actions, float* d_rewards, uint8_t* d_dones) {
  const uint32_t n = env->n;
  hipLaunchKernelGGL(k_env_step, dim3((n + 3) / 4), dim3(256), 0, env->stream, env->d_state, env->d_ep_steps, n,
                     d_actions, d_rewards, d_dones, env->acos_thr, env->d_flags);
  if (env->hashing)
    hipLaunchKernelGGL(k_env_raster<true>, dim3(n), dim3(256), 0, env->stream, env->d_state, n, env->d_obs, env->d_hash);
  else
    hipLaunchKernelGGL(k_env_raster<false>, dim3(n), dim3(256), 0, env->stream, env->d_state, n, env->d_obs, (uint64_t*)nullptr);
  QLX_HIP(hipGetLastError());
}

void env_launch_reset(qlx_env* env, const uint8_t* d_mask, int bump) {
  const uint32_t n = env->n;
  hipLaunchKernelGGL(k_env_reset, dim3(n), dim3(256), 0, env->stream, env->d_state, env->d_ep_steps, env->d_obs, n, env->seed,
                     env->id_offset, d_mask, bump);
  QLX_HIP(hipGetLastError());
}

}  // namespace qlx

using namespace qlx;

extern "C" {

int32_t qlx_env_action_space(int32_t kind) { return kind == QLX_ENV_BREAKOUT ? kActions : kind == QLX_ENV_BALLGAME ? 5 : -1; }
float qlx_env_reward_goal_mean(int32_t kind) {
  return kind == QLX_ENV_BREAKOUT ? (float)(kNumBricks - 1) : kind == QLX_ENV_BALLGAME ? 9.5f : -1.0f;
}

int32_t qlx_env_create(int32_t kind, uint32_t n_envs, uint64_t seed, int32_t device, qlx_env** out) {
  return guard([&] {
    QLX_CHECK(kind == QLX_ENV_BREAKOUT, QLX_E_INVALID, "unknown env kind");
    QLX_CHECK(n_envs > 0 && out, QLX_E_INVALID, "n_envs must be > 0");
    current_device_checked(device);
    auto* e = new qlx_env;
    try {   // a failure part-way releases what was built
      e->device = device;
      e->n = n_envs;
      e->seed = seed;
      e->acos_thr = acos_threshold_host();
      QLX_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
      QLX_HIP(hipMalloc(&e->d_state, sizeof(State) * n_envs));
      QLX_HIP(hipMalloc(&e->d_obs, (size_t)n_envs * kSlots * kFramePix));
      QLX_HIP(hipMalloc(&e->d_hash, sizeof(uint64_t) * n_envs));
      QLX_HIP(hipMalloc(&e->d_ep_steps, sizeof(uint32_t) * n_envs));
      QLX_HIP(hipMalloc(&e->d_flags, 16));
      QLX_HIP(hipMalloc(&e->d_tmp_u8, n_envs));
      QLX_HIP(hipMalloc(&e->d_tmp_u8b, n_envs));
      QLX_HIP(hipMalloc(&e->d_tmp_f32, sizeof(float) * n_envs));
      QLX_HIP(hipMemsetAsync(e->d_hash, 0, sizeof(uint64_t) * n_envs, e->stream));
      QLX_HIP(hipMemsetAsync(e->d_flags, 0, 16, e->stream));
      int8_t col[kFrame], row[kFrame];
      brick_luts(col, row);
      QLX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_brick_col), col, sizeof(col)));
      QLX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_brick_row), row, sizeof(row)));
      env_launch_reset(e, nullptr, 0);
      QLX_HIP(hipStreamSynchronize(e->stream));
    } catch (...) {
      qlx_env_destroy(e);
      throw;
    }
    *out = e;
  });
}

int32_t qlx_env_destroy(qlx_env* e) {
  return guard([&] {
    if (!e) return;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    (void)hipFree(e->d_state); (void)hipFree(e->d_obs); (void)hipFree(e->d_hash); (void)hipFree(e->d_flags);
    (void)hipFree(e->d_ep_steps);
    (void)hipFree(e->d_tmp_u8); (void)hipFree(e->d_tmp_u8b); (void)hipFree(e->d_tmp_f32); (void)hipFree(e->d_obs_view);
    if (e->own_stream) (void)hipStreamDestroy(e->stream);
    delete e;
  });
}

uint32_t qlx_env_count(const qlx_env* e) { return e ? e->n : 0; }

int32_t qlx_env_reset(qlx_env* e, const uint8_t* mask) {
  return guard([&] {
    QLX_CHECK(e, QLX_E_INVALID, "null env");
    QLX_HIP(hipSetDevice(e->device));
    if (mask) QLX_HIP(hipMemcpyAsync(e->d_tmp_u8, mask, e->n, hipMemcpyHostToDevice, e->stream));
    env_launch_reset(e, mask ? e->d_tmp_u8 : nullptr, 1);
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

int32_t qlx_env_step_dev(qlx_env* e, const uint8_t* d_actions, float* d_rewards, uint8_t* d_dones) {
  return guard([&] {
    QLX_CHECK(e && d_actions && d_rewards && d_dones, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    env_launch_step(e, d_actions, d_rewards, d_dones);
  });
}

int32_t qlx_env_step(qlx_env* e, const uint8_t* actions, float* rewards, uint8_t* dones) {
  return guard([&] {
    QLX_CHECK(e && actions && rewards && dones, QLX_E_INVALID, "null argument");
    for (uint32_t i = 0; i < e->n; ++i)
      QLX_CHECK(actions[i] < kActions, QLX_E_INVALID, "value out of range");   // Action::try_from_numeric
    QLX_HIP(hipSetDevice(e->device));
    QLX_HIP(hipMemcpyAsync(e->d_tmp_u8, actions, e->n, hipMemcpyHostToDevice, e->stream));
    env_launch_step(e, e->d_tmp_u8, e->d_tmp_f32, e->d_tmp_u8b);
    QLX_HIP(hipMemcpyAsync(rewards, e->d_tmp_f32, sizeof(float) * e->n, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipMemcpyAsync(dones, e->d_tmp_u8b, e->n, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

int32_t qlx_env_obs(qlx_env* e, uint8_t* out) {
  return guard([&] {
    QLX_CHECK(e && out, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    const size_t bytes = (size_t)e->n * kFramePix * kSlots;
    // (a device buffer kept by the env: the Rust Environment::step of INTEGRATION.md reads the state every step)
    if (!e->d_obs_view) QLX_HIP(hipMalloc(&e->d_obs_view, bytes));
    const size_t total = (size_t)e->n * kFramePix;
    hipLaunchKernelGGL(k_env_obs_view, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, e->stream, e->d_obs, e->n, e->d_obs_view);
    QLX_HIP(hipGetLastError());
    QLX_HIP(hipMemcpyAsync(out, e->d_obs_view, bytes, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

int32_t qlx_env_states(qlx_env* e, qlx_breakout_state* out) {
  return guard([&] {
    QLX_CHECK(e && out, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    QLX_HIP(hipMemcpyAsync(out, e->d_state, sizeof(State) * e->n, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

int32_t qlx_env_hashes(qlx_env* e, uint64_t* out) {
  return guard([&] {
    QLX_CHECK(e && out, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    QLX_HIP(hipMemcpyAsync(out, e->d_hash, sizeof(uint64_t) * e->n, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

int32_t qlx_env_sync(qlx_env* e) {
  return guard([&] {
    QLX_CHECK(e, QLX_E_INVALID, "null env");
    QLX_HIP(hipStreamSynchronize(e->stream));
    uint32_t flag = 0;
    QLX_HIP(hipMemcpy(&flag, e->d_flags, 4, hipMemcpyDeviceToHost));
    QLX_CHECK(flag == 0, QLX_E_INVALID, "action value out of range in a device step");
  });
}

}  // extern "C"
