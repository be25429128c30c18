// Learning statistics of the learner: the reference's learning_update_log
// (self_driving_tf_q_learner.rs:235-273) = DBSCAN clusters of the episode-reward history
// (src/ql/src/util/dbscan.rs:209-341, Display :91-133) + the action distribution over the replay + the
// episode / step / epsilon / reward-goal line.  Off the hot path: the action histogram runs on the device over
// the replay's action column (one byte per transition, HBM-bound, LDS-privatised bins); DBSCAN and the text are
// host code.
//
// DBSCAN on 1-D f32 values in O(n log n), exactly equal to the reference's generic O(n^2) expansion:
//  * |a - b| rounds monotonically, so every point's neighbourhood {j : |v_i - v_j| <= eps} is a contiguous
//    range of the value-sorted order (two pointers give all ranges);
//  * core points (range size > core_point_min_neighbors) connect iff some chain of cores within eps joins them,
//    and in sorted order that is "consecutive cores within eps": components are runs of cores;
//  * a component's members are the union of its cores' ranges = one sorted range; a point inside several
//    components' ranges (a border point) belongs to the component the reference forms first, i.e. the one
//    whose lowest core index is smallest (seeds are popped in index order and a component is only ever
//    started from its lowest-index core); everything else is noise;
//  * clusters are reported ordered by their lowest member index (cluster_analysis :250).
// Values and eps must be finite (eps >= 0): the reference's region query is undefined for NaN (its
// debug_assert requires a point to neighbour itself).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "objects.h"
#include "stats.h"

namespace qlx {

// ---------------- action histogram ----------------
__global__ __launch_bounds__(256) void k_action_counts(const uint8_t* actions, uint64_t len, uint32_t n_actions,
                                                       unsigned long long* counts) {
  __shared__ uint32_t bins[256];
  const uint32_t tid = threadIdx.x;
  bins[tid] = 0;
  __syncthreads();
  const uint64_t words = len / 16;
  const uint4* v = reinterpret_cast<const uint4*>(actions);
  for (uint64_t i = blockIdx.x * 256ull + tid; i < words; i += (uint64_t)gridDim.x * 256) {
    const uint4 w = v[i];
    const uint32_t parts[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(&bins[(parts[k] >> (8 * j)) & 0xFF], 1u);
  }
  if (blockIdx.x == 0)
    for (uint64_t i = words * 16 + tid; i < len; i += 256) atomicAdd(&bins[actions[i]], 1u);
  __syncthreads();
  if (tid < n_actions && bins[tid]) atomicAdd(&counts[tid], (unsigned long long)bins[tid]);
  // bytes >= n_actions cannot occur (actions are validated at every env step); count them in one spare bin
  if (tid >= n_actions && bins[tid]) atomicAdd(&counts[n_actions], (unsigned long long)bins[tid]);
}

void action_counts(hipStream_t s, const uint8_t* d_actions, uint64_t len, uint32_t n_actions, std::vector<uint64_t>& out) {
  QLX_CHECK(n_actions >= 1 && n_actions < 256, QLX_E_INVALID, "bad action space");
  unsigned long long* d = nullptr;
  QLX_HIP(hipMalloc(reinterpret_cast<void**>(&d), (n_actions + 1) * sizeof(unsigned long long)));
  QLX_HIP(hipMemsetAsync(d, 0, (n_actions + 1) * sizeof(unsigned long long), s));
  if (len) {
    const uint64_t blocks = std::min<uint64_t>(1024, std::max<uint64_t>(1, (len / 16 + 255) / 256));
    hipLaunchKernelGGL(k_action_counts, dim3((uint32_t)blocks), dim3(256), 0, s, d_actions, len, n_actions, d);
    QLX_HIP(hipGetLastError());
  }
  std::vector<unsigned long long> h(n_actions + 1);
  QLX_HIP(hipMemcpyAsync(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  QLX_HIP(hipStreamSynchronize(s));
  QLX_HIP(hipFree(d));
  QLX_CHECK(h[n_actions] == 0, QLX_E_STATE, "replay holds an action outside the action space");
  out.assign(h.begin(), h.begin() + n_actions);
}

// ---------------- DBSCAN (1-D, exact) ----------------
uint64_t dbscan_1d(const float* v, uint64_t n, float eps, uint64_t min_neighbors, int32_t* labels) {
  QLX_CHECK(std::isfinite(eps) && eps >= 0.0f, QLX_E_INVALID, "max_neighbor_distance must be finite and >= 0");
  for (uint64_t i = 0; i < n; ++i) QLX_CHECK(std::isfinite(v[i]), QLX_E_INVALID, "values must be finite");
  auto d = [](float a, float b) { return a >= b ? a - b : b - a; };
  std::vector<uint64_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) { return v[a] < v[b] || (v[a] == v[b] && a < b); });
  std::vector<uint64_t> lo(n), hi(n);
  for (uint64_t k = 0, l = 0, h = 0; k < n; ++k) {
    while (d(v[ord[k]], v[ord[l]]) > eps) ++l;
    if (h < k) h = k;
    while (h + 1 < n && d(v[ord[h + 1]], v[ord[k]]) <= eps) ++h;
    lo[k] = l;
    hi[k] = h;
  }
  // components: runs of sorted cores with consecutive gaps <= eps
  struct Comp { uint64_t first, last, seed; };   // sorted positions of the member range, lowest core index
  std::vector<Comp> comps;
  uint64_t prev_core = UINT64_MAX;
  for (uint64_t k = 0; k < n; ++k) {
    if (hi[k] - lo[k] + 1 <= min_neighbors) continue;
    if (prev_core != UINT64_MAX && d(v[ord[k]], v[ord[prev_core]]) <= eps) {
      Comp& c = comps.back();
      c.last = hi[k];
      c.seed = std::min(c.seed, ord[k]);
    } else {
      comps.push_back({lo[k], hi[k], ord[k]});
    }
    prev_core = k;
  }
  std::vector<uint64_t> by_seed(comps.size());
  std::iota(by_seed.begin(), by_seed.end(), 0);
  std::sort(by_seed.begin(), by_seed.end(), [&](uint64_t a, uint64_t b) { return comps[a].seed < comps[b].seed; });
  std::vector<int64_t> owner(n, -1);   // by original index
  for (uint64_t c : by_seed)
    for (uint64_t k = comps[c].first; k <= comps[c].last; ++k)
      if (owner[ord[k]] < 0) owner[ord[k]] = (int64_t)c;
  // report order: lowest member index
  std::vector<uint64_t> min_member(comps.size(), UINT64_MAX);
  for (uint64_t i = 0; i < n; ++i)
    if (owner[i] >= 0) min_member[owner[i]] = std::min(min_member[owner[i]], i);
  std::vector<uint64_t> rep(comps.size());
  std::iota(rep.begin(), rep.end(), 0);
  std::sort(rep.begin(), rep.end(), [&](uint64_t a, uint64_t b) { return min_member[a] < min_member[b]; });
  std::vector<int32_t> pos(comps.size());
  for (uint64_t r = 0; r < rep.size(); ++r) pos[rep[r]] = (int32_t)r;
  for (uint64_t i = 0; i < n; ++i) labels[i] = owner[i] < 0 ? -1 : pos[owner[i]];
  return comps.size();
}

static int fixed_digits(float eps) {   // Display's cluster_range precision ladder
  const float bounds[5] = {0.00001f, 0.0001f, 0.001f, 0.01f, 0.1f};
  for (int i = 0; i < 5; ++i)
    if (eps < bounds[i]) return 6 - i;
  return 1;
}

std::string dbscan_1d_text(const float* v, uint64_t n, float eps, uint64_t min_neighbors) {
  std::vector<int32_t> lab(n);
  const uint64_t nc = dbscan_1d(v, n, eps, min_neighbors, lab.data());
  struct C { uint64_t size = 0; float first = 0, lo = 0, hi = 0; bool seen = false; };
  std::vector<C> cs(nc);
  uint64_t noise = 0;
  for (uint64_t i = 0; i < n; ++i) {   // index order: the first member seen is the lowest index
    if (lab[i] < 0) { ++noise; continue; }
    C& c = cs[lab[i]];
    if (!c.seen) { c.seen = true; c.first = c.lo = c.hi = v[i]; }
    if (v[i] < c.lo) c.lo = v[i];          // first minimum
    if (!(v[i] < c.hi)) c.hi = v[i];       // last maximum
    ++c.size;
  }
  // clusters ordered by the value of their first member (stable: ties keep index order)
  std::stable_sort(cs.begin(), cs.end(), [](const C& a, const C& b) { return a.first < b.first; });
  const int p = fixed_digits(eps);
  std::string s;
  char buf[160];
  for (uint64_t k = 0; k < nc; ++k) {
    std::snprintf(buf, sizeof buf, "%s%llux(%.*f..%.*f)", k ? ", " : "", (unsigned long long)cs[k].size, p, (double)cs[k].lo, p,
                  (double)cs[k].hi);
    s += buf;
  }
  if (noise) {
    std::snprintf(buf, sizeof buf, ", %llux(noise)", (unsigned long long)noise);
    s += buf;
  }
  return s;
}

static std::string with_underscores(uint64_t x) {
  std::string digits = std::to_string(x);
  std::string out;
  const size_t lead = digits.size() % 3 == 0 ? 3 : digits.size() % 3;
  out.append(digits, 0, lead);
  for (size_t i = lead; i < digits.size(); i += 3) out += "_" + digits.substr(i, 3);
  return out;
}

std::string learning_log(const LogInputs& in) {
  QLX_CHECK(!in.rewards.empty(), QLX_E_STATE, "no finished episode yet (learning_update_log needs episode rewards)");
  const uint64_t nr = in.rewards.size();
  float sum = 0.0f;   // avg_episode_reward: sequential f32 sum / len
  for (float r : in.rewards) sum += r;
  const float avg = sum / (float)nr;
  const float low = *std::min_element(in.rewards.begin(), in.rewards.end());
  uint64_t total = 0;
  for (uint64_t c : in.counts) total += c;
  char head[512];
  std::snprintf(head, sizeof head,
                "\nepisode: %s, steps: %s, \xF0\x9D\x9B\xBE=%.2f, \xF0\x9D\x9C\x80=%.2f, reward_goal: {mean >= %.1f, low >= %.1f}, "
                "current_rewards: {mean: %.1f, low: %.1f}\nreward_distribution: ",
                with_underscores(in.episode_count).c_str(), with_underscores(in.step_count).c_str(), (double)in.gamma, in.epsilon,
                (double)in.goal_mean, (double)(in.goal_mean * in.goal_pct), (double)avg, (double)low);
  std::string s = head;
  s += dbscan_1d_text(in.rewards.data(), nr, 0.35f, nr / 30);
  s += "\naction_distribution (of last " + with_underscores(total) + "): ";
  bool first = true;
  for (size_t a = 0; a < in.counts.size(); ++a) {
    if (in.counts[a] == 0) continue;   // the reference's map only holds actions that occur
    const float ratio = 100.0f * (float)in.counts[a] / (float)total;
    char part[96];
    std::snprintf(part, sizeof part, "%s%s %.1f%%", first ? "" : ", ", in.action_names[a], (double)ratio);
    s += part;
    first = false;
  }
  return s;
}

int32_t copy_text(const std::string& s, char* buf, size_t cap, size_t* len) {
  if (len) *len = s.size();
  if (buf && cap) {
    const size_t k = std::min(cap - 1, s.size());
    std::memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return QLX_OK;
}

}  // namespace qlx

using namespace qlx;

extern "C" {

int32_t qlx_dbscan_f32(const float* values, uint64_t n, float max_neighbor_distance, uint64_t core_point_min_neighbors,
                       int32_t* labels, uint64_t* n_clusters) {
  return guard([&] {
    QLX_CHECK((values && labels) || n == 0, QLX_E_INVALID, "null argument");
    const uint64_t c = dbscan_1d(values, n, max_neighbor_distance, core_point_min_neighbors, labels);
    if (n_clusters) *n_clusters = c;
  });
}

int32_t qlx_dbscan_f32_format(const float* values, uint64_t n, float max_neighbor_distance, uint64_t core_point_min_neighbors,
                              char* buf, size_t cap, size_t* len) {
  return guard([&] {
    QLX_CHECK(values || n == 0, QLX_E_INVALID, "null argument");
    copy_text(dbscan_1d_text(values, n, max_neighbor_distance, core_point_min_neighbors), buf, cap, len);
  });
}

}  // extern "C"
