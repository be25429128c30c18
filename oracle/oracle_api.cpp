// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h header).
// Flat C interface of the CPU restatement for tests/oracle.py (ctypes). Never linked by the product.
#include <cmath>
#include <cstring>
#include <omp.h>

#include "breakout_ref.h"
#include "learner_ref.h"
#include "qnet_ref.h"
#include "rng_ref.h"

using namespace orc;

extern "C" {

struct OrcState {   // same field layout as qlx_breakout_state (include/qlx.h)
  float ball_x, ball_y, dir_x, dir_y;
  float panel_min_x, panel_min_y, panel_max_x, panel_max_y, panel_speed;
  uint32_t score, finished, next_slot, fault, reset_count;
  uint64_t bricks;
};

static void fill_state(const Env& e, OrcState* s) {
  const Mechanics& m = e.mech;
  s->ball_x = m.ball_center.x; s->ball_y = m.ball_center.y;
  s->dir_x = m.ball_dir.x; s->dir_y = m.ball_dir.y;
  s->panel_min_x = m.panel.min.x; s->panel_min_y = m.panel.min.y;
  s->panel_max_x = m.panel.max.x; s->panel_max_y = m.panel.max.y;
  s->panel_speed = m.panel_speed;
  s->score = m.score; s->finished = m.finished ? 1 : 0; s->next_slot = (uint32_t)e.next_slot;
  s->fault = (uint32_t)m.fault; s->reset_count = e.reset_count;
  uint64_t mask = 0;
  for (const auto& b : m.bricks) mask |= 1ull << b.id;
  s->bricks = mask;
}

// ---------------- RNG ----------------
void orc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) { philox4x32_10(ctr, key, out); }
void orc_stream_u32(uint64_t seed, uint32_t c1, uint32_t c2, uint32_t purpose, uint64_t start, int n, uint32_t* out) {
  Stream s(seed, c1, c2, purpose, start);
  for (int i = 0; i < n; ++i) out[i] = s.next_u32();
}
float orc_gen_range_f32(uint64_t seed, uint32_t c1, uint32_t c2, uint32_t purpose, float lo, float hi) {
  Stream s(seed, c1, c2, purpose);
  return gen_range_f32(s, lo, hi);
}
double orc_gen_f64_01(uint64_t seed, uint32_t c1, uint32_t c2, uint32_t purpose) {
  Stream s(seed, c1, c2, purpose);
  return gen_range_f64_01(s);
}
int orc_gen_u8(uint64_t seed, uint32_t c1, uint32_t c2, uint32_t purpose, uint64_t start, int n) {
  Stream s(seed, c1, c2, purpose, start);
  return gen_range_u8(s, (uint8_t)n);
}
void orc_sample_distinct(uint64_t seed, uint32_t update_idx, uint32_t rank, uint64_t len, int B, uint64_t* out) {
  generate_distinct_random_ids(seed, update_idx, rank, len, B, out);
}

// actions of the synthetic env-parity driver: Stream(action_seed, env, step, P_SYNTH) -> gen_range(0..3)
void orc_synth_actions(uint64_t action_seed, uint32_t n_envs, uint32_t step, uint8_t* out) {
  for (uint32_t e = 0; e < n_envs; ++e) {
    Stream sa(action_seed, e, step, P_SYNTH);
    out[e] = gen_range_u8(sa, 3);
  }
}

// ---------------- mechanics KATs ----------------
int orc_wall_left(float cx, float cy, float r, float mvx, float mvy, float* out) {
  ContactSurface cs; int fault = 0;
  const bool hit = wall_left({cx, cy}, r, {mvx, mvy}, &cs, &fault);
  if (hit) { out[0] = cs.way; out[1] = cs.approximation; out[2] = cs.normal.x; out[3] = cs.normal.y; }
  return hit ? 1 : 0;
}
int orc_wall_right(float cx, float cy, float r, float mvx, float mvy, float* out) {
  ContactSurface cs; int fault = 0;
  const bool hit = wall_right({cx, cy}, r, {mvx, mvy}, &cs, &fault);
  if (hit) { out[0] = cs.way; out[1] = cs.approximation; out[2] = cs.normal.x; out[3] = cs.normal.y; }
  return hit ? 1 : 0;
}
int orc_rect_check(float cx, float cy, float r, float mvx, float mvy, float x0, float y0, float x1, float y1, float* out) {
  ContactSurface cs;
  const bool hit = rect_check({cx, cy}, r, {mvx, mvy}, {{x0, y0}, {x1, y1}}, &cs);
  if (hit) { out[0] = cs.way; out[1] = cs.approximation; out[2] = cs.normal.x; out[3] = cs.normal.y; }
  return hit ? 1 : 0;
}
float orc_acos_threshold() { return acos_gt_half_pi_threshold(); }

// ---------------- single env ----------------
void* orc_env_new(uint64_t seed, uint32_t env_id) { auto* e = new Env; env_init(*e, seed, env_id); return e; }
void orc_env_free(void* h) { delete (Env*)h; }
void orc_env_reset(void* h) { env_reset(*(Env*)h); }
void orc_env_step(void* h, int action, float* reward, int* done) {
  bool d; env_step(*(Env*)h, action, reward, &d); *done = d ? 1 : 0;
}
void orc_env_state(void* h, OrcState* out) { fill_state(*(Env*)h, out); }
void orc_env_tensor(void* h, uint8_t* out) { env_state_tensor(*(Env*)h, out); }
void orc_env_frame(void* h, int slot, uint8_t* out_yx) { std::memcpy(out_yx, ((Env*)h)->frames[slot], kFramePix); }

// ---------------- batched env run (parity driver) ----------------
// Linear per-step hash (definition shared with the product's on-device checksum):
//   hf = sum_i img[i] * (i+1) * K1      over the new frame, i = y*84 + x
//   hs = sum_j f_j   * (j+1) * K2      over the state fields in OrcState order (floats as bits, +-0 -> 0)
//   H  = H * K3 + hf + hs               (all mod 2^64)
static const uint64_t K1 = 0x9E3779B97F4A7C15ull, K2 = 0xC2B2AE3D27D4EB4Full, K3 = 0x100000001B3ull;
static uint64_t fbits(float f) { if (f == 0.0f) return 0; uint32_t b; std::memcpy(&b, &f, 4); return b; }
static uint64_t state_hash(const OrcState& s) {
  const uint64_t f[15] = {fbits(s.ball_x), fbits(s.ball_y), fbits(s.dir_x), fbits(s.dir_y), fbits(s.panel_min_x),
                          fbits(s.panel_min_y), fbits(s.panel_max_x), fbits(s.panel_max_y), fbits(s.panel_speed),
                          s.score, s.finished, s.next_slot, s.fault, s.reset_count, s.bricks};
  uint64_t h = 0;
  for (int j = 0; j < 15; ++j) h += f[j] * ((uint64_t)(j + 1) * K2);
  return h;
}
static uint64_t frame_hash(const uint8_t* img) {
  uint64_t h = 0;
  for (int i = 0; i < kFramePix; ++i) h += (uint64_t)img[i] * ((uint64_t)(i + 1) * K1);
  return h;
}

// Runs n_envs envs for n_steps with actions from Stream(action_seed, env, step, P_SYNTH) (gen_range_u8(3)),
// resetting an env after done or max_steps_per_episode steps (as the learner does).
void orc_envs_run(uint64_t env_seed, uint32_t n_envs, uint32_t n_steps, uint64_t action_seed, uint64_t max_steps,
                  OrcState* final_states, uint64_t* hashes, float* total_reward, uint32_t* episodes,
                  uint8_t* final_tensors) {
#pragma omp parallel for schedule(dynamic, 4)
  for (uint32_t e = 0; e < n_envs; ++e) {
    Env env;
    env_init(env, env_seed, e);
    uint64_t H = 0, ep_steps = 0;
    float tot = 0.0f;
    uint32_t eps = 0;
    for (uint32_t t = 0; t < n_steps; ++t) {
      Stream sa(action_seed, e, t, P_SYNTH);
      const int a = gen_range_u8(sa, 3);
      float r; bool d;
      const int slot = env.next_slot;
      env_step(env, a, &r, &d);
      tot += r;
      ep_steps += 1;
      OrcState st; fill_state(env, &st);
      H = H * K3 + frame_hash(env.frames[slot]) + state_hash(st);
      if (d || ep_steps >= max_steps) { env_reset(env); ep_steps = 0; eps += 1; }
    }
    fill_state(env, &final_states[e]);
    hashes[e] = H;
    total_reward[e] = tot;
    episodes[e] = eps;
    if (final_tensors) env_state_tensor(env, final_tensors + (size_t)e * kStateBytes);
  }
}

// ---------------- Q-network ----------------
void* orc_qnet_new(uint64_t seed) { auto* q = new QNet; qnet_init_glorot(*q, seed); return q; }
void orc_qnet_free(void* h) { delete (QNet*)h; }
void orc_qnet_hparams(void* h, float* out) {   // lr, beta_1, beta_2, epsilon, clipnorm
  const QNet* q = (const QNet*)h;
  out[0] = q->lr; out[1] = q->beta1; out[2] = q->beta2; out[3] = q->eps; out[4] = q->clipnorm;
}
int orc_var_size(int v) { return kVarSize[v]; }
void orc_qnet_get(void* h, int var, int which, float* out) {
  QNet* q = (QNet*)h;
  const auto& src = which == 0 ? q->w[var] : which == 1 ? q->m[var] : q->v[var];
  std::memcpy(out, src.data(), src.size() * sizeof(float));
}
void orc_qnet_set(void* h, int var, int which, const float* in) {
  QNet* q = (QNet*)h;
  auto& dst = which == 0 ? q->w[var] : which == 1 ? q->m[var] : q->v[var];
  std::memcpy(dst.data(), in, dst.size() * sizeof(float));
}
int64_t orc_qnet_iterations(void* h) { return ((QNet*)h)->iterations; }
void orc_qnet_set_iterations(void* h, int64_t it) { ((QNet*)h)->iterations = it; }
void orc_qnet_forward(void* h, const uint8_t* x, int B, float* q, float* a1, float* a2, float* a3, float* a4) {
  Acts a;
  qnet_forward(*(QNet*)h, x, B, a);
  std::memcpy(q, a.q.data(), a.q.size() * 4);
  if (a1) std::memcpy(a1, a.a1.data(), a.a1.size() * 4);
  if (a2) std::memcpy(a2, a.a2.data(), a.a2.size() * 4);
  if (a3) std::memcpy(a3, a.a3.data(), a.a3.size() * 4);
  if (a4) std::memcpy(a4, a.a4.data(), a.a4.size() * 4);
}
// One train_model call: forward, Huber, backward, clip_by_norm + Adam. grads_out (raw grads, all vars
// concatenated) and norms_out are optional.
float orc_qnet_train(void* h, const uint8_t* x, const uint8_t* actions, const float* y, int B, float* grads_out,
                     float* norms_out) {
  QNet* q = (QNet*)h;
  Acts a;
  qnet_forward(*q, x, B, a);
  Grads g;
  const float loss = qnet_loss_backward(*q, x, actions, y, B, a, g);
  if (grads_out) {
    size_t off = 0;
    for (int v = 0; v < kNumVars; ++v) { std::memcpy(grads_out + off, g.g[v].data(), kVarSize[v] * 4); off += kVarSize[v]; }
  }
  qnet_apply_adam(*q, g, norms_out);
  return loss;
}

// the fp32 arithmetic of QLX_ARCH_NATURE_DQN (qnet32_ref.cpp)
void orc_qnet32_forward(void* h, const uint8_t* x, int B, float* q, float* a1, float* a2, float* a3, float* a4) {
  Acts a;
  qnet32_forward(*(QNet*)h, x, B, a);
  std::memcpy(q, a.q.data(), a.q.size() * 4);
  if (a1) std::memcpy(a1, a.a1.data(), a.a1.size() * 4);
  if (a2) std::memcpy(a2, a.a2.data(), a.a2.size() * 4);
  if (a3) std::memcpy(a3, a.a3.data(), a.a3.size() * 4);
  if (a4) std::memcpy(a4, a.a4.data(), a.a4.size() * 4);
}
void orc_qnet32_set_dense(int dense) { qnet32_set_dense(dense != 0); }
float orc_qnet32_train(void* h, const uint8_t* x, const uint8_t* actions, const float* y, int B, float* grads_out,
                       float* norms_out) {
  QNet* q = (QNet*)h;
  Acts a;
  qnet32_forward(*q, x, B, a);
  Grads g;
  const float loss = qnet32_loss_backward(*q, x, actions, y, B, a, g);
  if (grads_out) {
    size_t off = 0;
    for (int v = 0; v < kNumVars; ++v) { std::memcpy(grads_out + off, g.g[v].data(), kVarSize[v] * 4); off += kVarSize[v]; }
  }
  qnet32_apply_adam(*q, g, norms_out);
  return loss;
}
// clip_by_norm + Adam of the fp32 chain definition applied to given raw gradients (all variables concatenated) times
// scale, rounded once per element as the product does (learner.hip data parallel: the all-reduced sum times 1 / world,
// qnet32.hip k_norm32 / k_adam32); iterations += 1
void orc_qnet32_apply(void* h, const float* grads, float scale, float* norms_out) {
  Grads g;
  size_t off = 0;
  for (int v = 0; v < kNumVars; ++v) {
    g.g[v].resize(kVarSize[v]);
    for (int i = 0; i < kVarSize[v]; ++i) g.g[v][i] = grads[off + i] * scale;
    off += kVarSize[v];
  }
  qnet32_apply_adam(*(QNet*)h, g, norms_out);
}

// ---------------- learner ----------------
void* orc_learner_new(const LearnerParams* p) { return new Learner(*p); }
void orc_learner_free(void* h) { delete (Learner*)h; }
void orc_learner_vector_step(void* h) { ((Learner*)h)->vector_step(); }
void orc_learner_prefill(void* h, uint64_t n) { for (uint64_t i = 0; i < n; ++i) ((Learner*)h)->vector_step(false); }
uint64_t orc_learner_stats_events(void* h) { return ((Learner*)h)->stats_events; }
void* orc_learner_qnet(void* h, int which) { Learner* l = (Learner*)h; return which == 0 ? (void*)&l->online : (void*)&l->target; }
void orc_learner_counters(void* h, uint64_t* out /*[6]*/, double* eps, float* running_reward) {
  Learner* l = (Learner*)h;
  out[0] = l->step_count; out[1] = l->vec_steps; out[2] = l->update_count; out[3] = l->episode_count;
  out[4] = l->replay.len(); out[5] = l->solved() ? 1 : 0;
  *eps = l->epsilon; *running_reward = l->running_reward;
}
int orc_learner_last(void* h, uint8_t* actions, float* rewards, uint8_t* dones, float* losses, uint64_t* indices,
                     float* targets, float* q) {
  Learner* l = (Learner*)h;
  const size_t N = l->p.n_envs;
  if (actions) std::memcpy(actions, l->last_actions.data(), N);
  if (rewards) std::memcpy(rewards, l->last_rewards.data(), N * 4);
  if (dones) std::memcpy(dones, l->last_dones.data(), N);
  if (losses) std::memcpy(losses, l->last_losses.data(), l->last_losses.size() * 4);
  if (indices) std::memcpy(indices, l->last_indices.data(), l->last_indices.size() * 8);
  if (targets) std::memcpy(targets, l->last_targets.data(), l->last_targets.size() * 4);
  if (q && !l->last_q.empty()) std::memcpy(q, l->last_q.data(), l->last_q.size() * 4);
  return (int)l->last_losses.size();
}
void orc_learner_env_state(void* h, uint32_t e, OrcState* out) { fill_state(((Learner*)h)->envs[e], out); }
void orc_learner_env_tensor(void* h, uint32_t e, uint8_t* out) { std::memcpy(out, ((Learner*)h)->state[e]->data(), kStateBytes); }
// ReplayBuffer::get_many for logical indices (0 = oldest)
void orc_learner_replay_get(void* h, const uint64_t* idx, int B, uint8_t* s, uint8_t* s_next, uint8_t* a, float* r,
                            uint8_t* d) {
  Learner* l = (Learner*)h;
  for (int b = 0; b < B; ++b) {
    const Transition& t = l->replay.buf[idx[b]];
    if (s) std::memcpy(s + (size_t)b * kStateBytes, t.s->data(), kStateBytes);
    if (s_next) std::memcpy(s_next + (size_t)b * kStateBytes, t.s_next->data(), kStateBytes);
    if (a) a[b] = t.action;
    if (r) r[b] = t.reward;
    if (d) d[b] = t.done ? 1 : 0;
  }
}
// prioritized replay state: IS weights of the last vector step's batches, the sum tree's leaves [cap], per_max
void orc_learner_per(void* h, float* weights, float* leaves, float* per_max) {
  Learner* l = (Learner*)h;
  if (weights) std::memcpy(weights, l->last_weights.data(), l->last_weights.size() * 4);
  if (leaves) std::memcpy(leaves, l->tree.t.data() + l->tree.L, l->p.history_buffer_len * 4);
  if (per_max) *per_max = l->per_max;
}
// one prioritized draw per update u < U from a tree over the given leaves [cap] (physical slots)
void orc_per_sample(const float* leaves, uint64_t cap, uint64_t seed, uint32_t first_update, uint32_t n_updates, uint32_t rank,
                    uint64_t len, float beta, int B, uint64_t* slots, float* weights, float* total) {
  SumTree st(cap);
  for (uint64_t i = 0; i < cap; ++i) st.t[st.L + i] = leaves[i];
  for (size_t i = st.L - 1; i >= 1; --i) st.t[i] = st.t[2 * i] + st.t[2 * i + 1];
  if (total) *total = st.t[1];
  for (uint32_t u = 0; u < n_updates; ++u)
    per_sample(st, seed, first_update + u, rank, len, beta, B, slots + (size_t)u * B, weights + (size_t)u * B);
}
void orc_det_powf(const float* x, const float* y, uint64_t n, float* out) {
  for (uint64_t i = 0; i < n; ++i) out[i] = det_powf(x[i], y[i]);
}
size_t orc_learner_params_size() { return sizeof(LearnerParams); }
size_t orc_state_size() { return sizeof(OrcState); }
int orc_num_threads() { return omp_get_max_threads(); }

}  // extern "C"

// ---------------- BallGame (ballgame_ref.h) ----------------
#include "ballgame_ref.h"

extern "C" {

size_t orc_bg_state_size() { return sizeof(BgState); }
void orc_bg_initial_state(uint64_t seed, uint32_t env_id, uint32_t reset_count, BgState* out) {
  Stream s(seed, env_id, reset_count, P_BALLGAME);
  bg_random_initial_state(*out, s);
  out->reset_count = reset_count;
}
// Environment::step on a caller-held state (seed / id only matter for resets, which the caller drives)
void orc_bg_step(BgState* st, int action, float* reward, uint8_t* done) {
  BgEnv e;
  e.s = *st;
  e.seed = 0;
  e.id = 0;
  bool d;
  bg_env_step(e, (uint8_t)action, reward, &d);
  *st = e.s;
  *done = d ? 1 : 0;
}
void orc_bg_obs(const BgState* st, uint8_t* out) { bg_obs(*st, out); }
uint64_t orc_gen_range_usize_single(uint64_t seed, uint32_t c1, uint32_t c2, uint32_t purpose, uint64_t start, uint64_t n) {
  Stream s(seed, c1, c2, purpose, start);
  return gen_range_usize_single(s, n);
}

void* orc_bg_net_new(uint64_t seed) { auto* n = new BgNet; bg_net_init_glorot(*n, seed); return n; }
void orc_bg_net_free(void* h) { delete (BgNet*)h; }
void orc_bg_net_hparams(void* h, float* out) {
  const BgNet* n = (const BgNet*)h;
  out[0] = n->lr; out[1] = n->beta1; out[2] = n->beta2; out[3] = n->eps; out[4] = n->clipnorm;
}
int orc_bg_var_size(int v) { return kBgVarSize[v]; }
void orc_bg_net_get(void* h, int var, int which, float* out) {
  BgNet* n = (BgNet*)h;
  const auto& src = which == 0 ? n->w[var] : which == 1 ? n->m[var] : n->v[var];
  std::memcpy(out, src.data(), src.size() * sizeof(float));
}
void orc_bg_net_set(void* h, int var, int which, const float* in) {
  BgNet* n = (BgNet*)h;
  auto& dst = which == 0 ? n->w[var] : which == 1 ? n->m[var] : n->v[var];
  std::memcpy(dst.data(), in, dst.size() * sizeof(float));
}
void orc_bg_net_forward(void* h, const uint8_t* x, int B, float* q, float* a1, float* a2, float* a3) {
  BgActs a;
  bg_net_forward(*(BgNet*)h, x, B, a);
  std::memcpy(q, a.q.data(), a.q.size() * 4);
  if (a1) std::memcpy(a1, a.a1.data(), a.a1.size() * 4);
  if (a2) std::memcpy(a2, a.a2.data(), a.a2.size() * 4);
  if (a3) std::memcpy(a3, a.a3.data(), a.a3.size() * 4);
}
float orc_bg_net_train(void* h, const uint8_t* x, const uint8_t* actions, const float* y, int B, float* grads_out,
                       float* norms_out) {
  BgNet* n = (BgNet*)h;
  BgActs a;
  bg_net_forward(*n, x, B, a);
  BgGrads g;
  const float loss = bg_net_loss_backward(*n, x, actions, y, B, a, g);
  if (grads_out) {
    size_t off = 0;
    for (int v = 0; v < kBgVars; ++v) { std::memcpy(grads_out + off, g.g[v].data(), kBgVarSize[v] * 4); off += kBgVarSize[v]; }
  }
  bg_net_apply_adam(*n, g, norms_out);
  return loss;
}

void* orc_bg_learner_new(const BgParams* p) { return new BgLearner(*p); }
void orc_bg_learner_free(void* h) { delete (BgLearner*)h; }
void orc_bg_learner_vector_step(void* h) { ((BgLearner*)h)->vector_step(); }
void* orc_bg_learner_net(void* h, int which) { BgLearner* l = (BgLearner*)h; return which == 0 ? (void*)&l->online : (void*)&l->target; }
void orc_bg_learner_counters(void* h, uint64_t* out /*[6]*/, double* eps, float* running_reward) {
  BgLearner* l = (BgLearner*)h;
  out[0] = l->step_count; out[1] = l->vec_steps; out[2] = l->update_count; out[3] = l->episode_count;
  out[4] = l->replay.size(); out[5] = l->solved() ? 1 : 0;
  *eps = l->epsilon; *running_reward = l->running_reward;
}
int orc_bg_learner_last(void* h, uint8_t* actions, float* rewards, uint8_t* dones, float* losses, uint64_t* indices,
                        float* targets) {
  BgLearner* l = (BgLearner*)h;
  const size_t N = l->p.n_envs;
  if (actions) std::memcpy(actions, l->last_actions.data(), N);
  if (rewards) std::memcpy(rewards, l->last_rewards.data(), N * 4);
  if (dones) std::memcpy(dones, l->last_dones.data(), N);
  if (losses) std::memcpy(losses, l->last_losses.data(), l->last_losses.size() * 4);
  if (indices) std::memcpy(indices, l->last_indices.data(), l->last_indices.size() * 8);
  if (targets) std::memcpy(targets, l->last_targets.data(), l->last_targets.size() * 4);
  return (int)l->last_losses.size();
}
void orc_bg_learner_env_state(void* h, uint32_t e, BgState* out) { *out = ((BgLearner*)h)->envs[e].s; }
void orc_bg_learner_per(void* h, float* leaves, float* per_max) {   // sum-tree leaves [cap], per_max
  BgLearner* l = (BgLearner*)h;
  if (leaves) std::memcpy(leaves, l->tree.t.data() + l->tree.L, l->p.history_buffer_len * 4);
  if (per_max) *per_max = l->per_max;
}

}  // extern "C"
