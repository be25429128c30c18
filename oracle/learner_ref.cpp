// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h / learner_ref.h headers).
#include "learner_ref.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "rng_ref.h"

namespace orc {

void generate_distinct_random_ids(uint64_t seed, uint32_t update_idx, uint32_t rank, uint64_t len, int B, uint64_t* out) {
  // self_driving_tf_q_learner.rs:276-296: Uniform::from(0..len), reject values already drawn
  Stream s(seed, update_idx, rank, P_SAMPLE);
  const UniformUsize dist(len);
  for (int i = 0; i < B; ++i) {
    for (;;) {
      const uint64_t x = dist.sample(s);
      bool seen = false;
      for (int j = 0; j < i; ++j) if (out[j] == x) { seen = true; break; }
      if (!seen) { out[i] = x; break; }
    }
  }
}

float det_powf(float xf, float yf) {
  if (std::isnan(yf)) return NAN;   // a NaN exponent: NaN on both sides (no rint of NaN below)
  if (!(xf > 0.0f)) return xf == 0.0f ? (yf > 0.0f ? 0.0f : (yf < 0.0f ? INFINITY : 1.0f)) : NAN;
  if (std::isinf(xf)) return yf > 0.0f ? INFINITY : (yf < 0.0f ? 0.0f : 1.0f);
  int e = 0;
  double m = std::frexp((double)xf, &e);   // x = m 2^e, m in [0.5, 1) -> [sqrt(1/2), sqrt(2))
  if (m < 0.70710678118654752440) {
    m *= 2.0;
    e -= 1;
  }
  const double f = (m - 1.0) / (m + 1.0);
  const double s = f * f;
  double series = 1.0 / 23.0;   // sum_{i <= 11} s^i / (2 i + 1), Horner from the top term
  for (int i = 10; i >= 0; --i) series = std::fma(series, s, 1.0 / (double)(2 * i + 1));
  const double ln_x = std::fma((double)e, 0.69314718055994530942, (f * series) * 2.0);
  const double z = (double)yf * ln_x;
  if (z > 700.0) return INFINITY;
  if (z < -745.0) return 0.0f;
  const double k = std::rint(z * 1.44269504088896340736);   // z = k ln2 + r
  double r = std::fma(-k, 6.93147180369123816490e-01, z);
  r = std::fma(-k, 1.90821492927058770002e-10, r);
  double factorial = 1307674368000.0;   // 15!
  double poly = 1.0 / factorial;
  for (int i = 14; i >= 0; --i) {
    factorial = factorial / (double)(i + 1);
    poly = std::fma(poly, r, 1.0 / factorial);
  }
  return (float)std::ldexp(poly, (int)k);
}

void per_sample(const SumTree& st, uint64_t seed, uint32_t update_idx, uint32_t rank, uint64_t len, float beta, int B,
                uint64_t* slots, float* weights) {
  const float T = st.t[1];
  const float seg = T / (float)B;
  float wmax = 0.0f;
  for (int b = 0; b < B; ++b) {
    Stream s(seed, update_idx, rank, P_PER, (uint64_t)b);
    const float r = gen_range_f32(s, 0.0f, 1.0f);
    const float u = seg * ((float)b + r);
    slots[b] = st.find(u);
    const float p = st.t[st.L + slots[b]] / T;
    weights[b] = det_powf((float)len * p, -beta);
    wmax = std::max(wmax, weights[b]);
  }
  for (int b = 0; b < B; ++b) weights[b] = weights[b] / wmax;
}

// the Q-net arithmetic of the product under test: fp32 fmaf chains (qnet32_ref.cpp, bit-exact definition) or the
// double-accumulating restatement the bf16 product is held to within stated tolerances (qnet_ref.cpp)
void Learner::fwd(const QNet& q, const uint8_t* x, int B, Acts& a) const {
  if (p.qnet_precision == 0) qnet32_forward(q, x, B, a);
  else qnet_forward(q, x, B, a);
}

static StateRef snapshot(const Env& e) {   // Environment::state_as_rc / step_as_rc (prelude.rs:36,52-58)
  auto s = std::make_shared<std::vector<uint8_t>>(kStateBytes);
  env_state_tensor(e, s->data());
  return s;
}

Learner::Learner(const LearnerParams& prm) : p(prm), replay(prm.history_buffer_len), tree(prm.history_buffer_len) {
  envs.resize(p.n_envs);
  state.resize(p.n_envs);
  ep_reward.assign(p.n_envs, 0.0f);
  ep_steps.assign(p.n_envs, 0);
  for (uint32_t e = 0; e < p.n_envs; ++e) {
    env_init(envs[e], p.env_seed, e);
    state[e] = snapshot(envs[e]);
  }
  qnet_init_glorot(online, p.init_seed);
  target = online;   // stabilized_model: load_model_fn() again -> same initial weights (:107-108)
  epsilon = p.epsilon_max;
}

// Tensor<f32>::set(&[b, x, y, hist]) of the tensorflow crate: index from the dims with a bounds check per axis; the pixel
// from ImageBuffer::get_pixel(x, y) (bounds-checked, row-major y * width + x), loops hist / y / x as the reference nests
// them (breakout_environment.rs:63-74)
void Learner::pack_reference(const std::vector<StateRef>& states) {
  const uint64_t dims[4] = {(uint64_t)states.size(), (uint64_t)kFrame, (uint64_t)kFrame, (uint64_t)kSlots};
  std::vector<float> tensor((size_t)dims[0] * dims[1] * dims[2] * dims[3]);
  for (size_t b = 0; b < states.size(); ++b)
    for (int hist = 0; hist < kSlots; ++hist) {
      const uint8_t* v = states[b]->data();   // the u8 view [x][y][slot] holds each frame image's pixels
      for (uint32_t y = 0; y < (uint32_t)kFrame; ++y)
        for (uint32_t x = 0; x < (uint32_t)kFrame; ++x) {
          if (x >= (uint32_t)kFrame || y >= (uint32_t)kFrame) abort();   // get_pixel bounds
          const uint8_t pixel = v[((size_t)x * kFrame + y) * kSlots + hist];
          const uint64_t idx[4] = {b, x, y, (uint64_t)hist};
          uint64_t index = 0, d = 1;
          for (int i = 3; i >= 0; --i) {
            if (!(dims[i] > idx[i])) abort();
            index += idx[i] * d;
            d *= dims[i];
          }
          tensor[index] = (float)pixel;
        }
    }
  double s = 0.0;
  for (size_t i = 0; i < tensor.size(); i += 97) s += tensor[i];
  pack_sink += s;
}

void Learner::vector_step(bool train) {
  const uint32_t N = p.n_envs;
  last_actions.assign(N, 0);
  last_rewards.assign(N, 0.0f);
  last_dones.assign(N, 0);
  last_losses.clear();
  last_indices.clear();
  last_targets.clear();
  last_weights.clear();
  last_q.clear();
  const uint64_t step_before = step_count;
  // ---- acting (learn_episode :150-167) ----
  // greedy Q for every env that can be greedy in this vector step
  const bool any_greedy = step_count + N >= p.epsilon_pure_random_steps;
  if (any_greedy) {
    std::vector<uint8_t> x((size_t)N * kStateBytes);
    for (uint32_t e = 0; e < N; ++e) std::memcpy(&x[(size_t)e * kStateBytes], state[e]->data(), kStateBytes);
    if (pack_like_reference) pack_reference(state);   // to_multi_dim_array of each acting state (:36-53)
    Acts a;
    fwd(online, x.data(), (int)N, a);
    last_q = a.q;
  }
  const double interval = p.epsilon_max - p.epsilon_min;
  for (uint32_t e = 0; e < N; ++e) {
    step_count += 1;
    bool random = step_count < p.epsilon_pure_random_steps;
    if (!random) {
      Stream su(p.learner_seed, e, (uint32_t)vec_steps, P_ACT, 0);
      random = epsilon > gen_range_f64_01(su);
    }
    uint8_t a;
    if (random) {
      Stream sa(p.learner_seed, e, (uint32_t)vec_steps, P_ACT, 2);
      a = gen_range_u8(sa, kActions);
    } else {
      a = (uint8_t)argmax_first(&last_q[(size_t)e * kActions], kActions);
    }
    epsilon = std::max(epsilon - interval / p.epsilon_greedy_steps, p.epsilon_min);
    last_actions[e] = a;
  }
  // ---- env step + replay (learn_episode :169-178, :214-230) ----
  bool episode_ended = false;
  for (uint32_t e = 0; e < N; ++e) {
    float r; bool done;
    env_step(envs[e], last_actions[e], &r, &done);
    StateRef nxt = snapshot(envs[e]);
    ep_reward[e] += r;
    ep_steps[e] += 1;
    replay.add({last_actions[e], state[e], nxt, r, done});
    if (p.flags & 2u) tree.set(total_pushed % p.history_buffer_len, per_max);   // new transitions at max priority
    total_pushed += 1;
    state[e] = nxt;
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
      episode_ended = true;
      env_reset(envs[e]);
      state[e] = snapshot(envs[e]);
      ep_reward[e] = 0.0f;
      ep_steps[e] = 0;
    }
  }
  // ---- training updates (:181-202) ----
  const uint64_t triggers = step_count / p.update_after_actions - step_before / p.update_after_actions;
  if (train && replay.len() > p.batch_size && triggers > 0) {
    // every batch of the vector step is drawn from the replay (and priorities) as they stand after the pushes
    const int B = (int)p.batch_size;
    const uint64_t len = replay.len();
    std::vector<uint64_t> idx((size_t)triggers * B);
    std::vector<float> isw((size_t)triggers * B, 1.0f);
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
    std::vector<float> y((size_t)triggers * B);
    for (uint64_t t = 0; t < triggers; ++t) targets(&idx[t * B], &y[t * B]);
    for (uint64_t t = 0; t < triggers; ++t) update(&idx[t * B], (p.flags & 2u) ? &isw[t * B] : nullptr, &y[t * B]);
  }
  if (p.target_sync_steps > 0 && step_count / p.target_sync_steps != step_before / p.target_sync_steps)
    qnet_copy_weights(target, online);
  // statistics events (:204-212, :226-230): write_checkpoint + learning_update_log once per vector step that crossed a
  // multiple of stats_after_steps, and once more when an episode ended and the task is solved
  const uint64_t S = p.stats_after_steps;
  if (S > 0 && step_count / S != step_before / S) stats_events += 1;
  if (episode_ended && solved()) stats_events += 1;
  vec_steps += 1;
}

// Bellman targets of one sampled batch from the nets as they stand before the vector step's updates:
// y = r + gamma * max_a Q_target(s') (reference), or with double DQN r + gamma * Q_target(s', argmax_a Q_online(s'));
// y = r if done.  (Without double DQN this equals computing y inside each update: the target net does not move.)
void Learner::targets(const uint64_t* idx, float* y) const {
  const int B = (int)p.batch_size;
  std::vector<uint8_t> xn((size_t)B * kStateBytes);
  for (int b = 0; b < B; ++b) std::memcpy(&xn[(size_t)b * kStateBytes], replay.buf[idx[b]].s_next->data(), kStateBytes);
  if (pack_like_reference) {   // batch_to_multi_dim_array(state_next batch) (q_learning_model.rs:137)
    std::vector<StateRef> sn(B);
    for (int b = 0; b < B; ++b) sn[b] = replay.buf[idx[b]].s_next;
    const_cast<Learner*>(this)->pack_reference(sn);
  }
  Acts at;
  fwd(target, xn.data(), B, at);   // batch_predict_max_future_reward
  Acts an;
  if (p.flags & 1u) fwd(online, xn.data(), B, an);   // double DQN: the online net picks a*
  for (int b = 0; b < B; ++b) {
    const Transition& t = replay.buf[idx[b]];
    float v;
    if (p.flags & 1u) {
      v = at.q[(size_t)b * kActions + argmax_first(&an.q[(size_t)b * kActions], kActions)];
    } else {
      v = at.q[(size_t)b * kActions];
      for (int j = 1; j < kActions; ++j) v = std::max(v, at.q[(size_t)b * kActions + j]);
    }
    y[b] = t.reward + v * p.gamma;            // add_arrays(reward, array_mul(max_future, gamma))
    if (t.done) y[b] = t.reward;
  }
}

void Learner::update(const uint64_t* idx, const float* isw, const float* y) {
  const int B = (int)p.batch_size;
  std::vector<uint8_t> xs((size_t)B * kStateBytes), act(B);
  for (int b = 0; b < B; ++b) {   // ReplayBuffer::get_many
    const Transition& t = replay.buf[idx[b]];
    std::memcpy(&xs[(size_t)b * kStateBytes], t.s->data(), kStateBytes);
    act[b] = t.action;
  }
  if (pack_like_reference) {   // batch_to_multi_dim_array(state batch) (q_learning_model.rs:171)
    std::vector<StateRef> sb(B);
    for (int b = 0; b < B; ++b) sb[b] = replay.buf[idx[b]].s;
    pack_reference(sb);
  }
  Acts ao;
  fwd(online, xs.data(), B, ao);
  Grads g;
  std::vector<float> td(B);
  float loss;
  if (p.qnet_precision == 0) {
    loss = qnet32_loss_backward(online, xs.data(), act.data(), y, B, ao, g, isw, td.data());
    qnet32_apply_adam(online, g, nullptr);
  } else {
    loss = qnet_loss_backward(online, xs.data(), act.data(), y, B, ao, g, isw, td.data());
    qnet_apply_adam(online, g, nullptr);
  }
  if (p.flags & 2u) {   // new priorities (|td| + eps)^alpha, in batch order (a repeated slot keeps its last value)
    const uint64_t start = (total_pushed - replay.len()) % p.history_buffer_len;
    for (int b = 0; b < B; ++b) {
      const float pr = det_powf(td[b] + p.per_eps, p.per_alpha);
      tree.set((start + idx[b]) % p.history_buffer_len, pr);
      per_max = std::max(per_max, pr);
    }
  }
  last_losses.push_back(loss);
  last_indices.insert(last_indices.end(), idx, idx + B);
  last_targets.insert(last_targets.end(), y, y + B);
  last_weights.insert(last_weights.end(), isw ? isw : y, (isw ? isw : y) + B);
  if (!isw) std::fill(last_weights.end() - B, last_weights.end(), 1.0f);
  update_count += 1;
}

bool Learner::solved() const {   // :134-139
  if (episode_rewards.empty()) return false;
  // episode_reward_goal_mean (breakout_environment.rs:203-206), or the mocked goal
  const float goal = std::isnan(p.episode_reward_goal) ? (float)(kNumBricks - 1) : p.episode_reward_goal;
  float mn = episode_rewards.front();
  for (float v : episode_rewards) mn = std::min(mn, v);
  return running_reward >= goal && mn >= goal * p.lowest_episode_reward_goal_threshold_pct;
}

}  // namespace orc
