// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h header).  Never linked into the product.
//
// Restatement of the reference's learning-stats log, generic form, O(n^2):
//   DBSCAN          /root/reference/src/ql/src/util/dbscan.rs:209-341 cluster_analysis / region_query /
//                   build_cluster / append_new, for f32 elements with Distance = a - b or b - a (:24-37)
//   Display         dbscan.rs:91-133 "Yx(B..C), ..., Yx(noise)": clusters ordered by the value of their first
//                   (lowest-index) member under f32_cmp (:77-88), stable; range precision by max_neighbor_distance
//   log text        self_driving_tf_q_learner.rs:235-273 learning_update_log
// Pinned by the reference's own dbscan test vectors (dbscan.rs:370-376, tests/test_oracle_stats.py).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

namespace orc {

static float dist(float a, float b) { return a >= b ? a - b : b - a; }

static std::vector<size_t> region_query(const float* e, size_t n, size_t p, float eps) {
  std::vector<size_t> out;
  for (size_t i = 0; i < n; ++i)
    if (dist(e[p], e[i]) <= eps) out.push_back(i);
  return out;
}

struct Dbscan {
  std::vector<std::vector<size_t>> clusters;
  std::vector<size_t> noise;
};

static bool in_clusters(const Dbscan& r, size_t i) {
  for (const auto& c : r.clusters)
    if (std::find(c.begin(), c.end(), i) != c.end()) return true;
  return false;
}

Dbscan dbscan(const float* e, size_t n, float eps, size_t min_neighbors) {
  Dbscan r;
  std::deque<size_t> unvisited;
  for (size_t i = 0; i < n; ++i) unvisited.push_back(i);
  while (!unvisited.empty()) {
    const size_t p = unvisited.front();
    unvisited.pop_front();
    std::vector<size_t> neighbors = region_query(e, n, p, eps);
    if (neighbors.size() > min_neighbors) {   // build_cluster
      std::vector<size_t> forming{p};
      for (size_t k = 0; k < neighbors.size(); ++k) {
        const size_t pn = neighbors[k];
        auto it = std::lower_bound(unvisited.begin(), unvisited.end(), pn);
        if (it != unvisited.end() && *it == pn) {
          unvisited.erase(it);
          const std::vector<size_t> nn = region_query(e, n, pn, eps);
          if (nn.size() > min_neighbors)
            for (size_t x : nn)   // append_new
              if (std::find(neighbors.begin(), neighbors.end(), x) == neighbors.end()) neighbors.push_back(x);
        }
        if (std::find(forming.begin(), forming.end(), pn) == forming.end() && !in_clusters(r, pn)) {
          forming.push_back(pn);
          auto jt = std::lower_bound(r.noise.begin(), r.noise.end(), pn);
          if (jt != r.noise.end() && *jt == pn) r.noise.erase(jt);
        }
      }
      std::sort(forming.begin(), forming.end());
      r.clusters.push_back(forming);
    } else {
      r.noise.push_back(p);
    }
  }
  std::sort(r.clusters.begin(), r.clusters.end(),
            [](const std::vector<size_t>& a, const std::vector<size_t>& b) { return a.front() < b.front(); });
  return r;
}

static int f32_cmp(float a, float b) {   // dbscan.rs:77-88 (NaN orders first)
  if (a != a) return -1;
  if (b != b) return 1;
  if (a == b) return 0;
  return a < b ? -1 : 1;
}

std::string dbscan_format(const float* e, const Dbscan& r, float eps) {
  std::vector<size_t> order(r.clusters.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    return f32_cmp(e[r.clusters[a].front()], e[r.clusters[b].front()]) < 0;
  });
  const int prec = eps < 0.00001f ? 6 : eps < 0.0001f ? 5 : eps < 0.001f ? 4 : eps < 0.01f ? 3 : eps < 0.1f ? 2 : 1;
  std::string s;
  char buf[128];
  for (size_t i = 0; i < order.size(); ++i) {
    const auto& c = r.clusters[order[i]];
    // min_by / max_by under f32_cmp: first minimum, last maximum (Iterator::max_by keeps the last of equals)
    float lo = e[c[0]], hi = e[c[0]];
    for (size_t k : c) {
      if (f32_cmp(e[k], lo) < 0) lo = e[k];
      if (f32_cmp(e[k], hi) >= 0) hi = e[k];
    }
    if (i) s += ", ";
    std::snprintf(buf, sizeof buf, "%zux(%.*f..%.*f)", c.size(), prec, (double)lo, prec, (double)hi);
    s += buf;
  }
  if (!r.noise.empty()) {
    std::snprintf(buf, sizeof buf, ", %zux(noise)", r.noise.size());
    s += buf;
  }
  return s;
}

// num_format Grouping::Standard with separator "_"
static std::string grouped(uint64_t v) {
  std::string d = std::to_string(v), out;
  for (size_t i = 0; i < d.size(); ++i) {
    if (i && (d.size() - i) % 3 == 0) out += '_';
    out += d[i];
  }
  return out;
}

// learning_update_log; the action distribution lists actions in numeric order (the reference iterates an
// FxHashMap, whose order is not part of its contract) and skips actions never taken, as the map would
std::string update_log(uint64_t episode_count, uint64_t step_count, float gamma, double epsilon, float goal_mean, float pct,
                       const float* rewards, size_t n_rewards, const uint64_t* counts, int n_actions, const char* const* names) {
  const Dbscan r = dbscan(rewards, n_rewards, 0.35f, n_rewards / 30);
  float sum = 0.0f, mn = n_rewards ? rewards[0] : 0.0f;
  for (size_t i = 0; i < n_rewards; ++i) {
    sum += rewards[i];
    if (rewards[i] < mn) mn = rewards[i];
  }
  const float avg = n_rewards ? sum / (float)n_rewards : 0.0f;
  uint64_t total = 0;
  for (int a = 0; a < n_actions; ++a) total += counts[a];
  std::string actions;
  char buf[512];
  for (int a = 0; a < n_actions; ++a) {
    if (!counts[a]) continue;
    const float ratio = 100.0f * (float)counts[a] / (float)total;
    std::snprintf(buf, sizeof buf, "%s%s %.1f%%", actions.empty() ? "" : ", ", names[a], (double)ratio);
    actions += buf;
  }
  std::snprintf(buf, sizeof buf,
                "\nepisode: %s, steps: %s, \xF0\x9D\x9B\xBE=%.2f, \xF0\x9D\x9C\x80=%.2f, reward_goal: {mean >= %.1f, low >= %.1f}, "
                "current_rewards: {mean: %.1f, low: %.1f}\nreward_distribution: ",
                grouped(episode_count).c_str(), grouped(step_count).c_str(), (double)gamma, epsilon, (double)goal_mean,
                (double)(goal_mean * pct), (double)avg, (double)mn);
  std::string s = buf;
  s += dbscan_format(rewards, r, 0.35f);
  s += "\naction_distribution (of last " + grouped(total) + "): " + actions;
  return s;
}

}  // namespace orc

extern "C" {

// labels[i] = output position of i's cluster (clusters ordered by lowest member index) or -1 for noise
uint64_t orc_dbscan_f32(const float* e, uint64_t n, float eps, uint64_t min_neighbors, int32_t* labels) {
  const orc::Dbscan r = orc::dbscan(e, n, eps, min_neighbors);
  for (uint64_t i = 0; i < n; ++i) labels[i] = -1;
  for (size_t c = 0; c < r.clusters.size(); ++c)
    for (size_t i : r.clusters[c]) labels[i] = (int32_t)c;
  return r.clusters.size();
}

size_t orc_dbscan_f32_format(const float* e, uint64_t n, float eps, uint64_t min_neighbors, char* buf, size_t cap) {
  const std::string s = orc::dbscan_format(e, orc::dbscan(e, n, eps, min_neighbors), eps);
  if (cap) {
    const size_t k = std::min(cap - 1, s.size());
    std::memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return s.size();
}

size_t orc_update_log(uint64_t episode_count, uint64_t step_count, float gamma, double epsilon, float goal_mean, float pct,
                      const float* rewards, uint64_t n_rewards, const uint64_t* counts, int n_actions, int ballgame, char* buf,
                      size_t cap) {
  static const char* const kBreakout[] = {"None", "Left", "Right"};
  static const char* const kBallGame[] = {"\xE2\x86\x90", "\xE2\x86\x91", "\xE2\x86\x92", "\xE2\x86\x93", "o"};
  const std::string s = orc::update_log(episode_count, step_count, gamma, epsilon, goal_mean, pct, rewards, n_rewards, counts,
                                        n_actions, ballgame ? kBallGame : kBreakout);
  if (cap) {
    const size_t k = std::min(cap - 1, s.size());
    std::memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return s.size();
}

}  // extern "C"
