// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h / ballgame_ref.h headers).
#include "ballgame_ref.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace orc {

const int kBgVarSize[kBgVars] = {2 * 2 * 4 * 32, 32, 32 * 32, 32, 288 * 512, 512, 512 * 5, 5};

uint64_t gen_range_usize_single(Stream& s, uint64_t n) {
  // rand 0.8.5 src/distributions/uniform.rs UniformInt::sample_single_inclusive for u64 / usize
  const uint64_t range = n;
  const uint64_t zone = (range << __builtin_clzll(range)) - 1;
  for (;;) {
    const uint64_t v = s.next_u64();
    const unsigned __int128 m = (unsigned __int128)v * range;
    const uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    if (lo <= zone) return hi;
  }
}

void bg_random_initial_state(BgState& st, Stream& s) {
  // ballgame_test_environment.rs:100-123 (tuple fields are evaluated left to right)
  const uint8_t gx = (uint8_t)gen_range_usize_single(s, 3);
  const uint8_t bx = (uint8_t)gen_range_usize_single(s, 3);
  uint8_t ox, oy;
  for (;;) {
    ox = (uint8_t)gen_range_usize_single(s, 3);
    oy = (uint8_t)gen_range_usize_single(s, 3);
    const bool is_goal = ox == gx && oy == 0, is_ball = ox == bx && oy == 2, is_o1 = ox == 1 && oy == 1;
    if (!is_goal && !is_ball && !is_o1) break;
  }
  std::memset(st.field, BG_EMPTY, 9);
  st.field[gx * 3 + 0] = BG_GOAL;
  st.field[bx * 3 + 2] = BG_BALL;
  st.field[1 * 3 + 1] = BG_OBSTACLE;
  st.field[ox * 3 + oy] = BG_OBSTACLE;
  st.ball_x = bx;
  st.ball_y = 2;
  st.pad = 0;
  st.steps = 0;
}

void bg_env_init(BgEnv& e, uint64_t seed, uint32_t id) {
  e.seed = seed;
  e.id = id;
  e.s.reset_count = 0;
  Stream s(seed, id, 0, P_BALLGAME);
  bg_random_initial_state(e.s, s);
}

void bg_env_reset(BgEnv& e) {
  const uint32_t rc = e.s.reset_count + 1;
  Stream s(e.seed, e.id, rc, P_BALLGAME);
  bg_random_initial_state(e.s, s);
  e.s.reset_count = rc;
}

void bg_env_step(BgEnv& e, uint8_t action, float* reward, bool* done) {
  BgState& st = e.s;
  st.steps += 1;   // do_move (:155-190)
  const int x = st.ball_x, y = st.ball_y;
  auto valid = [&](int tx, int ty) {
    const uint8_t v = st.field[tx * 3 + ty];
    return v == BG_EMPTY || v == BG_GOAL;
  };
  int tx = -1, ty = -1;
  switch (action) {
    case 0: if (x > 0 && valid(x - 1, y)) { tx = x - 1; ty = y; } break;   // West
    case 1: if (y > 0 && valid(x, y - 1)) { tx = x; ty = y - 1; } break;   // North
    case 2: if (x < 2 && valid(x + 1, y)) { tx = x + 1; ty = y; } break;   // East
    case 3: if (y < 2 && valid(x, y + 1)) { tx = x; ty = y + 1; } break;   // South
    default: tx = x; ty = y; break;                                        // Nothing
  }
  const bool legal = tx >= 0;
  bool reached = false;
  if (legal) {
    reached = st.field[tx * 3 + ty] == BG_GOAL;
    st.field[x * 3 + y] = BG_EMPTY;
    st.field[tx * 3 + ty] = BG_BALL;
    st.ball_x = (uint8_t)tx;
    st.ball_y = (uint8_t)ty;
  }
  // Environment::step (:69-86)
  if (legal && reached) { *reward = 10.0f; *done = true; }
  else if (st.steps >= (uint32_t)kBgMaxSteps) { *reward = -10.0f; *done = true; }
  else if (legal) { *reward = -0.02f; *done = false; }
  else { *reward = -1.0f; *done = false; }
}

void bg_obs(const BgState& st, uint8_t* out) {
  std::memset(out, 0, kBgObs);
  for (int p = 0; p < 9; ++p) out[p * 4 + st.field[p]] = 1;
}

// ---------------- Q-model ----------------

void bg_net_init_glorot(BgNet& n, uint64_t seed) {
  const int fan_in[4] = {2 * 2 * 4, 32, 288, 512};
  const int fan_out[4] = {2 * 2 * 32, 32, 512, 5};
  for (int v = 0; v < kBgVars; ++v) {
    n.w[v].assign(kBgVarSize[v], 0.0f);
    n.m[v].assign(kBgVarSize[v], 0.0f);
    n.v[v].assign(kBgVarSize[v], 0.0f);
    if (v % 2 == 0) {
      const int l = v / 2;
      const float limit = std::sqrt(6.0f / (float)(fan_in[l] + fan_out[l]));
      Stream s(seed, (uint32_t)v, 1, P_INIT);
      for (int i = 0; i < kBgVarSize[v]; ++i) n.w[v][i] = gen_range_f32(s, -limit, limit);
    }
  }
  n.iterations = 0;
}

static inline float relu(float v) { return v > 0.0f ? v : 0.0f; }

void bg_net_forward(const BgNet& n, const uint8_t* x, int B, BgActs& a) {
  a.a1.assign((size_t)B * 288, 0.0f);
  a.a2.assign((size_t)B * 288, 0.0f);
  a.a3.assign((size_t)B * 512, 0.0f);
  a.q.assign((size_t)B * 5, 0.0f);
  const float *k0 = n.w[0].data(), *b0 = n.w[1].data(), *k1 = n.w[2].data(), *b1 = n.w[3].data();
  const float *k2 = n.w[4].data(), *b2 = n.w[5].data(), *k3 = n.w[6].data(), *b3 = n.w[7].data();
  for (int b = 0; b < B; ++b) {
    const uint8_t* xb = x + (size_t)b * kBgObs;
    float* a1 = &a.a1[(size_t)b * 288];
    float* a2 = &a.a2[(size_t)b * 288];
    float* a3 = &a.a3[(size_t)b * 512];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int o = 0; o < 32; ++o) {   // 'same' 2x2: taps past the edge read the zero padding
          double s = 0.0;
          for (int di = 0; di < 2; ++di)
            for (int dj = 0; dj < 2; ++dj) {
              if (i + di > 2 || j + dj > 2) continue;
              for (int c = 0; c < 4; ++c)
                s += (double)xb[((i + di) * 3 + j + dj) * 4 + c] * (double)k0[((di * 2 + dj) * 4 + c) * 32 + o];
            }
          a1[(i * 3 + j) * 32 + o] = relu((float)s + b0[o]);
        }
    for (int p = 0; p < 9; ++p)
      for (int o = 0; o < 32; ++o) {
        double s = 0.0;
        for (int c = 0; c < 32; ++c) s += (double)a1[p * 32 + c] * (double)k1[c * 32 + o];
        a2[p * 32 + o] = relu((float)s + b1[o]);
      }
    for (int u = 0; u < 512; ++u) {   // Flatten (i, j, c) = a2 as stored
      double s = 0.0;
      for (int k = 0; k < 288; ++k) s += (double)a2[k] * (double)k2[k * 512 + u];
      a3[u] = relu((float)s + b2[u]);
    }
    for (int q = 0; q < 5; ++q) {
      double s = 0.0;
      for (int u = 0; u < 512; ++u) s += (double)a3[u] * (double)k3[u * 5 + q];
      a.q[(size_t)b * 5 + q] = (float)s + b3[q];
    }
  }
}

float bg_net_loss_backward(const BgNet& n, const uint8_t* x, const uint8_t* actions, const float* y, int B, const BgActs& a,
                           BgGrads& g, const float* weights, float* td_abs) {
  for (int v = 0; v < kBgVars; ++v) g.g[v].assign(kBgVarSize[v], 0.0f);
  const float *k1 = n.w[2].data(), *k2 = n.w[4].data(), *k3 = n.w[6].data();
  // MSE (mean over the batch) of e = q_a - y: dL/dq_a = 2 e / B
  std::vector<float> dq((size_t)B * 5, 0.0f);
  double loss = 0.0;
  for (int b = 0; b < B; ++b) {
    const float e = a.q[(size_t)b * 5 + actions[b]] - y[b];
    const float w = weights ? weights[b] : 1.0f;   // prioritized-replay IS weight
    loss += (double)w * ((double)e * (double)e);
    dq[(size_t)b * 5 + actions[b]] = 2.0f * (w * e) / (float)B;
    if (td_abs) td_abs[b] = std::fabs(e);
  }
  std::vector<float> dz3((size_t)B * 512), dz2((size_t)B * 288), dz1((size_t)B * 288);
  for (int u = 0; u < 512; ++u)
    for (int q = 0; q < 5; ++q) {
      double s = 0.0;
      for (int b = 0; b < B; ++b) s += (double)a.a3[(size_t)b * 512 + u] * (double)dq[(size_t)b * 5 + q];
      g.g[6][u * 5 + q] = (float)s;
    }
  for (int q = 0; q < 5; ++q) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += dq[(size_t)b * 5 + q];
    g.g[7][q] = (float)s;
  }
  for (int b = 0; b < B; ++b)
    for (int u = 0; u < 512; ++u) {
      double s = 0.0;
      for (int q = 0; q < 5; ++q) s += (double)dq[(size_t)b * 5 + q] * (double)k3[u * 5 + q];
      dz3[(size_t)b * 512 + u] = a.a3[(size_t)b * 512 + u] > 0.0f ? (float)s : 0.0f;
    }
  for (int k = 0; k < 288; ++k)
    for (int u = 0; u < 512; ++u) {
      double s = 0.0;
      for (int b = 0; b < B; ++b) s += (double)a.a2[(size_t)b * 288 + k] * (double)dz3[(size_t)b * 512 + u];
      g.g[4][k * 512 + u] = (float)s;
    }
  for (int u = 0; u < 512; ++u) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += dz3[(size_t)b * 512 + u];
    g.g[5][u] = (float)s;
  }
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < 288; ++k) {
      double s = 0.0;
      for (int u = 0; u < 512; ++u) s += (double)dz3[(size_t)b * 512 + u] * (double)k2[k * 512 + u];
      dz2[(size_t)b * 288 + k] = a.a2[(size_t)b * 288 + k] > 0.0f ? (float)s : 0.0f;
    }
  for (int c = 0; c < 32; ++c)
    for (int o = 0; o < 32; ++o) {
      double s = 0.0;
      for (int b = 0; b < B; ++b)
        for (int p = 0; p < 9; ++p) s += (double)a.a1[(size_t)b * 288 + p * 32 + c] * (double)dz2[(size_t)b * 288 + p * 32 + o];
      g.g[2][c * 32 + o] = (float)s;
    }
  for (int o = 0; o < 32; ++o) {
    double s = 0.0;
    for (int b = 0; b < B; ++b)
      for (int p = 0; p < 9; ++p) s += dz2[(size_t)b * 288 + p * 32 + o];
    g.g[3][o] = (float)s;
  }
  for (int b = 0; b < B; ++b)
    for (int p = 0; p < 9; ++p)
      for (int c = 0; c < 32; ++c) {
        double s = 0.0;
        for (int o = 0; o < 32; ++o) s += (double)dz2[(size_t)b * 288 + p * 32 + o] * (double)k1[c * 32 + o];
        dz1[(size_t)b * 288 + p * 32 + c] = a.a1[(size_t)b * 288 + p * 32 + c] > 0.0f ? (float)s : 0.0f;
      }
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int c = 0; c < 4; ++c)
        for (int o = 0; o < 32; ++o) {
          double s = 0.0;
          for (int b = 0; b < B; ++b)
            for (int i = 0; i + di < 3; ++i)
              for (int j = 0; j + dj < 3; ++j)
                s += (double)x[(size_t)b * kBgObs + ((i + di) * 3 + j + dj) * 4 + c] * (double)dz1[(size_t)b * 288 + (i * 3 + j) * 32 + o];
          g.g[0][((di * 2 + dj) * 4 + c) * 32 + o] = (float)s;
        }
  for (int o = 0; o < 32; ++o) {
    double s = 0.0;
    for (int b = 0; b < B; ++b)
      for (int p = 0; p < 9; ++p) s += dz1[(size_t)b * 288 + p * 32 + o];
    g.g[1][o] = (float)s;
  }
  return (float)(loss / (double)B);
}

void bg_net_apply_adam(BgNet& n, const BgGrads& g, float* norms_out) {
  // identical to qnet_apply_adam (legacy keras Adam: clip_by_norm per variable + ResourceApplyAdam)
  const float t = (float)(n.iterations + 1);
  const float b1p = std::pow(n.beta1, t), b2p = std::pow(n.beta2, t);
  const float alpha = n.lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
  for (int v = 0; v < kBgVars; ++v) {
    double ss = 0.0;
    for (float x : g.g[v]) ss += (double)x * (double)x;
    const float l2sum = (float)ss;
    const float l2norm = l2sum > 0.0f ? std::sqrt(l2sum) : l2sum;
    if (norms_out) norms_out[v] = l2norm;
    const float denom = std::max(l2norm, n.clipnorm);
    for (int i = 0; i < kBgVarSize[v]; ++i) {
      const float gc = (g.g[v][i] * n.clipnorm) / denom;
      n.m[v][i] += (gc - n.m[v][i]) * (1.0f - n.beta1);
      n.v[v][i] += (gc * gc - n.v[v][i]) * (1.0f - n.beta2);
      n.w[v][i] -= (n.m[v][i] * alpha) / (std::sqrt(n.v[v][i]) + n.eps);
    }
  }
  n.iterations += 1;
}

// ---------------- learner ----------------

void generate_distinct_random_ids(uint64_t seed, uint32_t update_idx, uint32_t rank, uint64_t len, int B, uint64_t* out);
int argmax_first(const float* q, int n);

BgLearner::BgLearner(const BgParams& prm) : p(prm), tree(prm.history_buffer_len) {
  envs.resize(p.n_envs);
  ep_reward.assign(p.n_envs, 0.0f);
  ep_steps.assign(p.n_envs, 0);
  for (uint32_t e = 0; e < p.n_envs; ++e) bg_env_init(envs[e], p.env_seed, p.rank * p.n_envs + e);
  bg_net_init_glorot(online, p.init_seed);
  target = online;
  epsilon = p.epsilon_max;
}

void BgLearner::vector_step() {   // learner_ref.cpp vector_step over BallGame
  const uint32_t N = p.n_envs;
  last_actions.assign(N, 0);
  last_rewards.assign(N, 0.0f);
  last_dones.assign(N, 0);
  last_losses.clear();
  last_indices.clear();
  last_targets.clear();
  const uint64_t step_before = step_count;
  std::vector<float> q;
  if (step_count + N >= p.epsilon_pure_random_steps) {
    std::vector<uint8_t> x((size_t)N * kBgObs);
    for (uint32_t e = 0; e < N; ++e) bg_obs(envs[e].s, &x[(size_t)e * kBgObs]);
    BgActs a;
    bg_net_forward(online, x.data(), (int)N, a);
    q = a.q;
  }
  const double interval = p.epsilon_max - p.epsilon_min;
  for (uint32_t e = 0; e < N; ++e) {
    step_count += 1;
    bool random = step_count < p.epsilon_pure_random_steps;
    const uint32_t gid = p.rank * N + e;
    if (!random) {
      Stream su(p.learner_seed, gid, (uint32_t)vec_steps, P_ACT, 0);
      random = epsilon > gen_range_f64_01(su);
    }
    uint8_t a;
    if (random) {
      Stream sa(p.learner_seed, gid, (uint32_t)vec_steps, P_ACT, 2);
      a = gen_range_u8(sa, kBgActions);
    } else {
      a = (uint8_t)argmax_first(&q[(size_t)e * kBgActions], kBgActions);
    }
    epsilon = std::max(epsilon - interval / p.epsilon_greedy_steps, p.epsilon_min);
    last_actions[e] = a;
  }
  for (uint32_t e = 0; e < N; ++e) {
    BgTransition t;
    t.action = last_actions[e];
    t.s = envs[e].s;
    float r;
    bool done;
    bg_env_step(envs[e], last_actions[e], &r, &done);
    t.s_next = envs[e].s;
    t.reward = r;
    t.done = done;
    if (replay.size() >= p.history_buffer_len) replay.pop_front();
    replay.push_back(t);
    if (p.flags & 2u) tree.set(total_pushed % p.history_buffer_len, per_max);   // new transitions at max priority
    total_pushed += 1;
    ep_reward[e] += r;
    ep_steps[e] += 1;
    last_rewards[e] = r;
    last_dones[e] = done ? 1 : 0;
    if (done || ep_steps[e] >= p.max_steps_per_episode) {
      episode_rewards.push_back(ep_reward[e]);
      if (episode_rewards.size() > p.episode_reward_history_buffer_len) episode_rewards.pop_front();
      if (episode_count >= p.episode_reward_history_buffer_len) {
        float s = 0.0f;
        for (float v : episode_rewards) s += v;
        running_reward = s / (float)episode_rewards.size();
      }
      episode_count += 1;
      bg_env_reset(envs[e]);
      ep_reward[e] = 0.0f;
      ep_steps[e] = 0;
    }
  }
  const uint64_t triggers = step_count / p.update_after_actions - step_before / p.update_after_actions;
  if (replay.size() > p.batch_size && triggers > 0) {   // all batches sampled and targeted up front (learner_ref.cpp)
    const int B = (int)p.batch_size;
    const uint64_t len = replay.size();
    std::vector<uint64_t> idx((size_t)triggers * B);
    std::vector<float> isw((size_t)triggers * B, 1.0f), y((size_t)triggers * B);
    for (uint64_t t = 0; t < triggers; ++t) {
      if (p.flags & 2u) {
        const uint64_t start = (total_pushed - len) % p.history_buffer_len;
        std::vector<uint64_t> slots(B);
        per_sample(tree, p.learner_seed, (uint32_t)(update_count + t), p.rank, len, p.per_beta, B, slots.data(), &isw[t * B]);
        for (int b = 0; b < B; ++b) idx[t * B + b] = (slots[b] + p.history_buffer_len - start) % p.history_buffer_len;
      } else {
        generate_distinct_random_ids(p.learner_seed, (uint32_t)(update_count + t), p.rank, len, B, &idx[t * B]);
      }
    }
    for (uint64_t t = 0; t < triggers; ++t) targets(&idx[t * B], &y[t * B]);
    for (uint64_t t = 0; t < triggers; ++t) update(&idx[t * B], (p.flags & 2u) ? &isw[t * B] : nullptr, &y[t * B]);
  }
  if (p.target_sync_steps > 0 && step_count / p.target_sync_steps != step_before / p.target_sync_steps)
    for (int v = 0; v < kBgVars; ++v) target.w[v] = online.w[v];
  vec_steps += 1;
}

// y = r + gamma max_a Q_target(s') (or, double DQN, r + gamma Q_target(s', argmax_a Q_online(s'))); r if done
void BgLearner::targets(const uint64_t* idx, float* y) const {
  const int B = (int)p.batch_size;
  std::vector<uint8_t> xn((size_t)B * kBgObs);
  for (int b = 0; b < B; ++b) bg_obs(replay[idx[b]].s_next, &xn[(size_t)b * kBgObs]);
  BgActs at, an;
  bg_net_forward(target, xn.data(), B, at);
  if (p.flags & 1u) bg_net_forward(online, xn.data(), B, an);
  for (int b = 0; b < B; ++b) {
    const BgTransition& t = replay[idx[b]];
    float v;
    if (p.flags & 1u) {
      v = at.q[(size_t)b * 5 + argmax_first(&an.q[(size_t)b * 5], 5)];
    } else {
      v = at.q[(size_t)b * 5];
      for (int j = 1; j < 5; ++j) v = std::max(v, at.q[(size_t)b * 5 + j]);
    }
    y[b] = t.done ? t.reward : t.reward + v * p.gamma;
  }
}

void BgLearner::update(const uint64_t* idx, const float* isw, const float* y) {
  const int B = (int)p.batch_size;
  std::vector<uint8_t> xs((size_t)B * kBgObs), act(B);
  for (int b = 0; b < B; ++b) {
    const BgTransition& t = replay[idx[b]];
    bg_obs(t.s, &xs[(size_t)b * kBgObs]);
    act[b] = t.action;
  }
  BgActs ao;
  bg_net_forward(online, xs.data(), B, ao);
  BgGrads g;
  std::vector<float> td(B);
  const float loss = bg_net_loss_backward(online, xs.data(), act.data(), y, B, ao, g, isw, td.data());
  bg_net_apply_adam(online, g, nullptr);
  if (p.flags & 2u) {   // (|td| + eps)^alpha per drawn slot, the last draw wins
    const uint64_t start = (total_pushed - replay.size()) % p.history_buffer_len;
    for (int b = 0; b < B; ++b) {
      const float pr = det_powf(td[b] + p.per_eps, p.per_alpha);
      tree.set((start + idx[b]) % p.history_buffer_len, pr);
      per_max = std::max(per_max, pr);
    }
  }
  last_losses.push_back(loss);
  last_indices.insert(last_indices.end(), idx, idx + B);
  last_targets.insert(last_targets.end(), y, y + B);
  update_count += 1;
}

bool BgLearner::solved() const {   // self_driving_tf_q_learner.rs:134-139 with goal 9.5
  if (episode_rewards.empty()) return false;
  const float goal = 9.5f;
  float mn = episode_rewards.front();
  for (float v : episode_rewards) mn = std::min(mn, v);
  return running_reward >= goal && mn >= goal * p.lowest_episode_reward_goal_threshold_pct;
}

}  // namespace orc
