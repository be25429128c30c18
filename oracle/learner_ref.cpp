// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h / learner_ref.h headers).
#include "learner_ref.h"

#include <algorithm>
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

static StateRef snapshot(const Env& e) {   // Environment::state_as_rc / step_as_rc (prelude.rs:36,52-58)
  auto s = std::make_shared<std::vector<uint8_t>>(kStateBytes);
  env_state_tensor(e, s->data());
  return s;
}

Learner::Learner(const LearnerParams& prm) : p(prm), replay(prm.history_buffer_len) {
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

void Learner::vector_step() {
  const uint32_t N = p.n_envs;
  last_actions.assign(N, 0);
  last_rewards.assign(N, 0.0f);
  last_dones.assign(N, 0);
  last_losses.clear();
  last_indices.clear();
  last_targets.clear();
  last_q.clear();
  const uint64_t step_before = step_count;
  // ---- acting (learn_episode :150-167) ----
  // greedy Q for every env that can be greedy in this vector step
  const bool any_greedy = step_count + N >= p.epsilon_pure_random_steps;
  if (any_greedy) {
    std::vector<uint8_t> x((size_t)N * kStateBytes);
    for (uint32_t e = 0; e < N; ++e) std::memcpy(&x[(size_t)e * kStateBytes], state[e]->data(), kStateBytes);
    Acts a;
    qnet_forward(online, x.data(), (int)N, a);
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
  for (uint32_t e = 0; e < N; ++e) {
    float r; bool done;
    env_step(envs[e], last_actions[e], &r, &done);
    StateRef nxt = snapshot(envs[e]);
    ep_reward[e] += r;
    ep_steps[e] += 1;
    replay.add({last_actions[e], state[e], nxt, r, done});
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
      env_reset(envs[e]);
      state[e] = snapshot(envs[e]);
      ep_reward[e] = 0.0f;
      ep_steps[e] = 0;
    }
  }
  // ---- training updates (:181-202) ----
  const uint64_t triggers = step_count / p.update_after_actions - step_before / p.update_after_actions;
  if (replay.len() > p.batch_size)
    for (uint64_t t = 0; t < triggers; ++t) update();
  if (p.target_sync_steps > 0 && step_count / p.target_sync_steps != step_before / p.target_sync_steps)
    qnet_copy_weights(target, online);
  vec_steps += 1;
}

void Learner::update() {
  const int B = (int)p.batch_size;
  std::vector<uint64_t> idx(B);
  generate_distinct_random_ids(p.learner_seed, (uint32_t)update_count, p.rank, replay.len(), B, idx.data());
  std::vector<uint8_t> xs((size_t)B * kStateBytes), xn((size_t)B * kStateBytes), act(B);
  std::vector<float> rew(B), y(B);
  std::vector<uint8_t> dn(B);
  for (int b = 0; b < B; ++b) {   // ReplayBuffer::get_many
    const Transition& t = replay.buf[idx[b]];
    std::memcpy(&xs[(size_t)b * kStateBytes], t.s->data(), kStateBytes);
    std::memcpy(&xn[(size_t)b * kStateBytes], t.s_next->data(), kStateBytes);
    act[b] = t.action; rew[b] = t.reward; dn[b] = t.done ? 1 : 0;
  }
  Acts at;
  qnet_forward(target, xn.data(), B, at);   // batch_predict_max_future_reward
  for (int b = 0; b < B; ++b) {
    float mx = at.q[(size_t)b * kActions];
    for (int j = 1; j < kActions; ++j) mx = std::max(mx, at.q[(size_t)b * kActions + j]);
    y[b] = rew[b] + mx * p.gamma;            // add_arrays(reward, array_mul(max_future, gamma))
    if (dn[b]) y[b] = rew[b];
  }
  Acts ao;
  qnet_forward(online, xs.data(), B, ao);
  Grads g;
  const float loss = qnet_loss_backward(online, xs.data(), act.data(), y.data(), B, ao, g);
  qnet_apply_adam(online, g, nullptr);
  last_losses.push_back(loss);
  last_indices.insert(last_indices.end(), idx.begin(), idx.end());
  last_targets.insert(last_targets.end(), y.begin(), y.end());
  update_count += 1;
}

bool Learner::solved() const {   // :134-139
  if (episode_rewards.empty()) return false;
  const float goal = (float)(kNumBricks - 1);   // episode_reward_goal_mean (breakout_environment.rs:203-206)
  float mn = episode_rewards.front();
  for (float v : episode_rewards) mn = std::min(mn, v);
  return running_reward >= goal && mn >= goal * p.lowest_episode_reward_goal_threshold_pct;
}

}  // namespace orc
