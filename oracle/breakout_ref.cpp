// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h header).  Restates mechanics.rs et al.
// Each function cites the reference lines it follows.
#include "breakout_ref.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "rng_ref.h"

namespace orc {

// ---- constants: mechanics.rs:12-44 -------------------------------------------------
static constexpr float GRID_X = 600.0f, GRID_Y = 600.0f;
static constexpr float CEILING_Y = 0.0f;
static constexpr float SPACE_GRANULARITY = 0.001f;
static const float TIME_GRANULARITY = 20000000.0f / 1000000000.0f;   // Duration::as_secs_f32(20ms)
static constexpr float PANEL_LEN_X = 60.0f, PANEL_LEN_Y = 10.0f;
static constexpr float PANEL_CENTER_Y = GRID_Y - 30.0f;
static constexpr float PANEL_MAX_SPEED = 160.0f;
static constexpr float PANEL_ACCEL = 20.0f;
static constexpr float PANEL_SLOWDOWN = 7.0f;
static constexpr float BRICK_EDGE = 25.0f;
static constexpr float BRICK_SPACING = 2.0f;
static constexpr int BRICK_ROWS = 3;
static constexpr float BALL_RADIUS = 10.0f;
static constexpr float BRICKS_LEFT = BALL_RADIUS * 3.0f;
static constexpr float BRICKS_RIGHT_MIN = BRICKS_LEFT;
static constexpr float BRICKS_FIRST_TOP = 60.0f;
static constexpr float BALL_SPEED = 200.0f;
static constexpr float CONTACT_PREDICTION = 0.8f;
static constexpr float PENETRATION_LIMIT = 0.0f;
static constexpr float FRAC_PI_2_F = 1.57079637050628662109375f;   // std::f32::consts::FRAC_PI_2
static constexpr int MAX_RECURSION = 64;
static constexpr int MAX_BSEARCH = 64;

// ---- emath 0.22 Vec2 ---------------------------------------------------------------
static inline V2 vadd(V2 a, V2 b) { return {a.x + b.x, a.y + b.y}; }
static inline V2 vsub(V2 a, V2 b) { return {a.x - b.x, a.y - b.y}; }
static inline V2 vmul(V2 a, float s) { return {a.x * s, a.y * s}; }
static inline V2 vdiv(V2 a, float s) { return {a.x / s, a.y / s}; }
static inline V2 vneg(V2 a) { return {-a.x, -a.y}; }
static inline float vdot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
// Vec2::length = self.x.hypot(self.y) -> glibc 2.35 __ieee754_hypotf:
// (float) sqrt((double)x*x + (double)y*y) for finite inputs.
static inline float vlen(V2 a) {
  if (!std::isfinite(a.x) || !std::isfinite(a.y)) return std::hypot(a.x, a.y);
  return (float)std::sqrt((double)a.x * (double)a.x + (double)a.y * (double)a.y);
}
static inline V2 vnormalized(V2 a) {
  const float l = vlen(a);
  if (l <= 0.0f) return a;
  return vdiv(a, l);
}

// algebra_2d.rs:47-53  r = v - 2 (v . n) n
static inline V2 reflected_vector(V2 v, V2 n) { return vsub(v, vmul(n, 2.0f * vdot(v, n))); }
// algebra_2d.rs:55-61  acos(normalized(v1) . normalized(v2))
static inline float vector_angle(V2 v1, V2 v2) { return std::acos(vdot(vnormalized(v1), vnormalized(v2))); }

float acos_gt_half_pi_threshold() {
  // Largest f32 d with acosf(d) > FRAC_PI_2 is found by scanning negative floats near 0:
  // acosf is monotone decreasing, so acosf(d) > FRAC_PI_2  <=>  d < T  with T = the
  // smallest float for which acosf(T) <= FRAC_PI_2.  Exported so tests can check the
  // product's constant against glibc.
  float d = -1e-5f;
  while (std::acos(d) > FRAC_PI_2_F) d = std::nextafter(d, 1.0f);
  return d;
}

// ---- parry2d 0.13.8: query::contact(Ball at c, Cuboid around AABB) ----------------------
struct Contact { float dist; V2 normal1; V2 normal2; };

// Aabb::project_local_point_and_get_feature (local frame: mins = -he, maxs = he).
static void project_local_point(V2 he, V2 p, V2* proj, bool* is_inside, int* face_axis, bool* face_min) {
  const float mins_pt[2] = {-he.x - p.x, -he.y - p.y};
  const float pt_maxs[2] = {p.x - he.x, p.y - he.y};
  const float shift[2] = {std::max(mins_pt[0], 0.0f) - std::max(pt_maxs[0], 0.0f),
                          std::max(mins_pt[1], 0.0f) - std::max(pt_maxs[1], 0.0f)};
  const bool inside = shift[0] == 0.0f && shift[1] == 0.0f;
  if (!inside) {
    *proj = {p.x + shift[0], p.y + shift[1]};
    *is_inside = false;
    // feature: the non-zero shift axis (edge) or a vertex; only used on the degenerate branch
    *face_axis = shift[0] != 0.0f ? 0 : 1;
    *face_min = shift[*face_axis] > 0.0f;
    return;
  }
  float best = -FLT_MAX;
  int best_id = 0;
  for (int i = 0; i < 2; ++i) {
    if (mins_pt[i] < pt_maxs[i]) {
      if (pt_maxs[i] > best) { best_id = i + 1; best = pt_maxs[i]; }
    } else if (mins_pt[i] > best) {
      best_id = -(i + 1); best = mins_pt[i];
    }
  }
  float s[2] = {0.0f, 0.0f};
  if (best_id < 0) { s[-best_id - 1] = best; *face_axis = -best_id - 1; *face_min = true; }
  else { s[best_id - 1] = -best; *face_axis = best_id - 1; *face_min = false; }
  *proj = {p.x + s[0], p.y + s[1]};
  *is_inside = true;
}

// contact_ball_convex_polyhedron -> contact_convex_polyhedron_ball(pos12.inverse(), cuboid, ball)
// then Contact::swapped().  Translation-only isometries: the identity rotations leave every
// component unchanged (up to the sign of an exact zero, which no later comparison observes).
static bool contact_test_circle_aabb(V2 c, float r, const AABB& bb, Contact* out) {
  const V2 bc = {(bb.min.x + bb.max.x) / 2.0f, (bb.min.y + bb.max.y) / 2.0f};   // AaBB::center
  const V2 he = {(bb.max.x - bb.min.x) / 2.0f, (bb.max.y - bb.min.y) / 2.0f};
  const V2 t12 = vsub(bc, c);          // pos1.inv_mul(pos2).translation
  const V2 center = vneg(t12);         // (pos12.inverse()).translation = ball centre in cuboid frame
  V2 proj; bool inside; int fax; bool fmin;
  project_local_point(he, center, &proj, &inside, &fax, &fmin);
  const V2 d = vsub(proj, center);
  const float sq = d.x * d.x + d.y * d.y;   // nalgebra norm_squared (dotx special case for 2-vectors)
  float dist; V2 n1;
  if (sq > FLT_EPSILON * FLT_EPSILON) {     // Unit::try_new_and_get(v, DEFAULT_EPSILON)
    const float len = std::sqrt(sq);
    const V2 dir = vdiv(d, len);
    if (inside) { dist = -len - r; n1 = dir; }
    else { dist = len - r; n1 = vneg(dir); }
  } else {
    // Degenerate branch: the ball centre lies on the cuboid boundary (proj == centre).
    // parry2d takes the feature normal there; a centre exactly on a corner gets the vertex
    // normal (diagonal).  This is what the reference KAT mechanics.rs:721 (way 2.07, normal
    // (1,1)/sqrt2 for a ball ending exactly on the corner) requires, so it pins this branch.
    dist = -r;
    const float sx = center.x >= he.x - FLT_EPSILON ? 1.0f : (center.x <= -he.x + FLT_EPSILON ? -1.0f : 0.0f);
    const float sy = center.y >= he.y - FLT_EPSILON ? 1.0f : (center.y <= -he.y + FLT_EPSILON ? -1.0f : 0.0f);
    if (sx != 0.0f && sy != 0.0f) n1 = vdiv({sx, sy}, std::sqrt(sx * sx + sy * sy));
    else if (sx != 0.0f || sy != 0.0f) n1 = {sx, sy};
    else n1 = {0.0f, 1.0f};
    (void)fax; (void)fmin;
  }
  if (dist <= CONTACT_PREDICTION) {
    out->dist = dist;
    out->normal1 = vneg(n1);   // ball-side normal (swapped contact), points towards the cuboid
    out->normal2 = n1;         // cuboid outward normal, points towards the ball
    return true;
  }
  return false;
}

// ---- mechanics.rs:260-315 wall tests ------------------------------------------------
bool wall_left(V2 center, float radius, V2 mv, ContactSurface* out, int* fault) {
  const float wdx = center.x - radius;
  if (!(wdx >= 0.0f)) *fault |= F_WALL_ASSERT;
  if (wdx + mv.x > 0.0f) return false;
  const V2 way = vmul(mv, wdx / std::fabs(mv.x));
  *out = {vlen(way), 0.0f, {1.0f, 0.0f}};
  return true;
}
bool wall_right(V2 center, float radius, V2 mv, ContactSurface* out, int* fault) {
  const float wdx = GRID_X - center.x - radius;
  if (!(wdx >= 0.0f)) *fault |= F_WALL_ASSERT;
  if (mv.x < wdx) return false;
  const V2 way = vmul(mv, wdx / std::fabs(mv.x));
  *out = {vlen(way), 0.0f, {-1.0f, 0.0f}};
  return true;
}
static bool wall_top(V2 center, float radius, V2 mv, ContactSurface* out, int* fault) {
  const float wdy = center.y - radius - CEILING_Y;
  if (!(wdy >= 0.0f)) *fault |= F_WALL_ASSERT;
  if (wdy + mv.y > 0.0f) return false;
  const V2 way = vmul(mv, wdy / std::fabs(mv.y));
  *out = {vlen(way), 0.0f, {0.0f, 1.0f}};
  return true;
}

// ---- mechanics.rs:337-443 find_non_penetrating_collision ---------------------------------
static ContactSurface binary_search_first_contact(V2 c, float r, V2 mv, float lo, float hi, const AABB& bb,
                                                  int depth, int* fault) {
  // mechanics.rs:361-389, recursion unrolled into a loop
  for (;;) {
    if (depth > MAX_BSEARCH) { *fault |= F_RECURSION; return {vlen(mv) * hi, 0.0f, {0.0f, 1.0f}}; }
    const float m = (lo + hi) / 2.0f;
    Contact ct;
    const bool hit = contact_test_circle_aabb(vadd(c, vmul(mv, m)), r, bb, &ct);
    if (!hit) { lo = m; }
    else if (ct.dist < -PENETRATION_LIMIT) { hi = m; }
    else return {vlen(mv) * m, ct.dist, ct.normal2};
    ++depth;
  }
}

static bool find_non_penetrating_collision(V2 c, float r, V2 mv, const AABB& bb, ContactSurface* out, int* fault) {
  Contact ct;
  if (!contact_test_circle_aabb(vadd(c, mv), r, bb, &ct)) return false;
  if (ct.dist < -PENETRATION_LIMIT) {
    // moved_distance_after_collision(p, n1, mv) = p / (n1 . mv / |mv|)   (:351-358)
    const float x = std::fabs(ct.dist) / (vdot(ct.normal1, mv) / vlen(mv));
    const float portion = 1.0f - x / vlen(mv);
    Contact ct2;
    const bool hit2 = contact_test_circle_aabb(vadd(c, vmul(mv, portion)), r, bb, &ct2);
    if (!hit2) { *out = binary_search_first_contact(c, r, mv, portion, 1.0f, bb, 0, fault); return true; }
    if (ct2.dist < -PENETRATION_LIMIT) { *out = binary_search_first_contact(c, r, mv, 0.0f, portion, bb, 0, fault); return true; }
    *out = {vlen(mv) * portion, ct2.dist, ct2.normal2};
    return true;
  }
  *out = {vlen(mv), ct.dist, ct.normal2};
  return true;
}

// mechanics.rs:317-335
bool rect_check(V2 center, float radius, V2 mv, AABB rect, ContactSurface* out) {
  int fault = 0;
  ContactSurface cs;
  if (!find_non_penetrating_collision(center, radius, mv, rect, &cs, &fault)) return false;
  if (std::fabs(vector_angle(mv, cs.normal)) > FRAC_PI_2_F) { *out = cs; return true; }
  return false;
}

// ---- mechanics.rs:485-539 ContactCandidates -------------------------------------------
struct Candidate { ContactSurface s; int brick_idx; };   // brick_idx = index into bricks vector, -1 = none

static void candidates_consider(std::vector<Candidate>& v, const Candidate& c, int* fault) {
  if (!(c.s.approximation >= -PENETRATION_LIMIT && c.s.approximation <= CONTACT_PREDICTION)) *fault |= F_CANDIDATE_ASSERT;
  v.push_back(c);
  if (v.size() > 1) {
    float shortest = INFINITY;
    for (const auto& e : v) { const float len = e.s.way + e.s.approximation; if (len < shortest) shortest = len; }
    std::vector<Candidate> kept;
    for (const auto& e : v) if (e.s.way + e.s.approximation <= shortest + SPACE_GRANULARITY) kept.push_back(e);
    v.swap(kept);
  }
}

static bool effective_collision_surface(const std::vector<Candidate>& v, ContactSurface* out) {
  if (v.empty()) return false;
  if (v.size() == 1) { *out = v[0].s; return true; }
  V2 n = {0.0f, 0.0f};
  for (const auto& e : v) n = vadd(n, e.s.normal);
  n = vnormalized(n);
  float dist = 0.0f, way = 0.0f;
  for (const auto& e : v) dist = dist + e.s.approximation;
  dist = dist / (float)v.size();
  for (const auto& e : v) way = way + e.s.way;
  way = way / (float)v.size();
  *out = {way, dist, n};
  return true;
}

// ---- mechanics.rs:186-213 check_collisions ----------------------------------------------
static std::vector<Candidate> check_collisions(const Mechanics& m, V2 mv, int* fault) {
  std::vector<Candidate> cands;
  ContactSurface cs;
  if (wall_left(m.ball_center, m.ball_radius, mv, &cs, fault)) candidates_consider(cands, {cs, -1}, fault);
  if (wall_right(m.ball_center, m.ball_radius, mv, &cs, fault)) candidates_consider(cands, {cs, -1}, fault);
  if (wall_top(m.ball_center, m.ball_radius, mv, &cs, fault)) candidates_consider(cands, {cs, -1}, fault);
  if (rect_check(m.ball_center, m.ball_radius, mv, m.panel, &cs)) candidates_consider(cands, {cs, -1}, fault);
  for (size_t i = 0; i < m.bricks.size(); ++i)
    if (rect_check(m.ball_center, m.ball_radius, mv, m.bricks[i].shape, &cs)) candidates_consider(cands, {cs, (int)i}, fault);
  return cands;
}

// ---- mechanics.rs:137-184 proceed_ball_with (recursion -> loop) --------------------------
static void proceed_ball_with(Mechanics& m, V2 mv) {
  for (int depth = 0;; ++depth) {
    if (vlen(mv) < SPACE_GRANULARITY) return;
    if (depth > MAX_RECURSION) { m.fault |= F_RECURSION; return; }
    std::vector<Candidate> cands = check_collisions(m, mv, &m.fault);
    std::vector<int> hit;
    for (const auto& c : cands) if (c.brick_idx >= 0) hit.push_back(c.brick_idx);
    std::sort(hit.begin(), hit.end());
    for (auto it = hit.rbegin(); it != hit.rend(); ++it) {
      m.bricks.erase(m.bricks.begin() + *it);
      m.score += 1;
    }
    ContactSurface col;
    if (effective_collision_surface(cands, &col)) {
      const V2 collision_center = vadd(m.ball_center, vmul(m.ball_dir, col.way));
      const float remaining = vlen(mv) - col.way;
      const V2 refl = vnormalized(reflected_vector(m.ball_dir, col.normal));
      m.ball_center = collision_center;
      m.ball_dir = refl;
      const V2 rem_mv = vmul(refl, remaining);
      if (vlen(rem_mv) > 0.0f) { mv = rem_mv; continue; }
      return;
    }
    m.ball_center = vadd(m.ball_center, mv);
    return;
  }
}

// ---- mechanics.rs:612-649 speed helpers ------------------------------------------------
static inline float granulate_speed(float s) { return std::round(s * 1000.0f) / 1000.0f; }
static inline float decrease_speed(float s, float brk) {
  if (s > 0.0f) return std::max(granulate_speed(s - brk), 0.0f);
  if (s < 0.0f) return std::max(granulate_speed(s + brk), 0.0f);   // sign quirk (:624) kept
  return 0.0f;
}
static inline float accelerate(float s, float a, float limit) {
  const float v = s + a;
  float r;
  if (std::fabs(v) > limit) r = std::signbit(v) ? -limit : limit;
  else r = v;
  return granulate_speed(r);
}

// ---- mechanics.rs:56-116 construction ----------------------------------------------------
void mechanics_init(Mechanics& m, uint64_t seed, uint32_t env_id, uint32_t reset_count) {
  m.bricks.clear();
  int id = 0;
  for (int row = 0; row < BRICK_ROWS; ++row) {
    float left_x = BRICKS_LEFT;
    const float upper_y = BRICKS_FIRST_TOP + (float)row * (BRICK_EDGE + BRICK_SPACING);
    for (;;) {
      const AABB b = {{left_x, upper_y - BRICK_EDGE}, {left_x + BRICK_EDGE, upper_y}};
      if (b.max.x >= GRID_X - BRICKS_RIGHT_MIN) break;
      left_x = b.max.x + BRICK_SPACING;
      m.bricks.push_back({b, id++});
    }
  }
  Stream s(seed, env_id, reset_count, P_BALL);
  m.ball_center = {GRID_X * 0.5f, GRID_Y * 0.5f};
  m.ball_radius = BALL_RADIUS;
  m.ball_dir = {gen_range_f32(s, -0.35f, -0.15f), -1.0f};   // :103
  m.ball_speed = BALL_SPEED;
  m.panel = {{GRID_X / 2.0f - PANEL_LEN_X / 2.0f, PANEL_CENTER_Y - PANEL_LEN_Y / 2.0f},
             {GRID_X / 2.0f + PANEL_LEN_X / 2.0f, PANEL_CENTER_Y + PANEL_LEN_Y / 2.0f}};
  m.panel_speed = 0.0f;
  m.finished = false;
  m.score = 0;
  m.fault = 0;
}

// mechanics.rs:119-135, 553-588
void mechanics_time_step(Mechanics& m, int action) {
  // Panel::proceed
  const float dx = m.panel_speed * TIME_GRANULARITY;
  AABB pot = {{m.panel.min.x + dx, m.panel.min.y + 0.0f}, {m.panel.max.x + dx, m.panel.max.y + 0.0f}};
  if (pot.min.x <= 0.0f) {
    const float t = -pot.min.x;
    m.panel = {{pot.min.x + t, pot.min.y + 0.0f}, {pot.max.x + t, pot.max.y + 0.0f}};
    m.panel_speed = 0.0f;
  } else if (pot.max.x >= GRID_X) {
    const float t = GRID_X - pot.max.x;
    m.panel = {{pot.min.x + t, pot.min.y + 0.0f}, {pot.max.x + t, pot.max.y + 0.0f}};
    m.panel_speed = 0.0f;
  } else {
    m.panel = pot;
  }
  // Ball::move_vector (:258)
  const V2 mv = vmul(vmul(vnormalized(m.ball_dir), m.ball_speed), TIME_GRANULARITY);
  proceed_ball_with(m, mv);
  // check_game_end_situation (:131-135)
  if (m.ball_center.y >= m.panel.max.y || m.bricks.empty()) m.finished = true;
  if (!m.finished) {
    if (action == 0) m.panel_speed = decrease_speed(m.panel_speed, PANEL_SLOWDOWN);
    else if (action == 1) m.panel_speed = accelerate(m.panel_speed, -PANEL_ACCEL, PANEL_MAX_SPEED);
    else m.panel_speed = accelerate(m.panel_speed, PANEL_ACCEL, PANEL_MAX_SPEED);
  }
}

// ---- build-defined rasterizer ----------------------------------------------------------
// Pixel (px, py) samples world point ((px+0.5)*S, (py+0.5)*S), S = 600/84.  Half-open AABB
// coverage; disk coverage for the ball; paint order background < bricks < panel < ball.
static void fill_rect(uint8_t* img, const float* w, const AABB& b, uint8_t v) {
  // coverage is separable: pixel covered iff its x sample and its y sample are inside
  for (int py = 0; py < kFrame; ++py) {
    if (!(b.min.y <= w[py] && w[py] < b.max.y)) continue;
    for (int px = 0; px < kFrame; ++px)
      if (b.min.x <= w[px] && w[px] < b.max.x) img[py * kFrame + px] = v;
  }
}

void rasterize(const Mechanics& m, uint8_t* img) {
  const float S = 600.0f / 84.0f;
  float w[kFrame];
  for (int p = 0; p < kFrame; ++p) w[p] = ((float)p + 0.5f) * S;
  std::memset(img, 0, kFramePix);
  for (const auto& b : m.bricks) fill_rect(img, w, b.shape, kLumaBrick);
  fill_rect(img, w, m.panel, kLumaPanel);
  const float rr = m.ball_radius * m.ball_radius;
  for (int py = 0; py < kFrame; ++py) {
    const float ddy = w[py] - m.ball_center.y;
    for (int px = 0; px < kFrame; ++px) {
      const float ddx = w[px] - m.ball_center.x;
      if (ddx * ddx + ddy * ddy <= rr) img[py * kFrame + px] = kLumaBall;
    }
  }
}

// ---- BreakoutEnvironment ----------------------------------------------------------------
void env_init(Env& e, uint64_t seed, uint32_t env_id) {
  e.seed = seed; e.env_id = env_id; e.reset_count = 0;
  mechanics_init(e.mech, seed, env_id, 0);
  std::memset(e.frames, 0, sizeof(e.frames));
  e.next_slot = 0;
}

void env_reset(Env& e) {
  e.reset_count += 1;
  mechanics_init(e.mech, e.seed, e.env_id, e.reset_count);
  std::memset(e.frames, 0, sizeof(e.frames));   // FrameRingBuffer::new
  e.next_slot = 0;
}

void env_step(Env& e, int action, float* reward, bool* done) {
  const uint32_t prev = e.mech.score;
  mechanics_time_step(e.mech, action);
  rasterize(e.mech, e.frames[e.next_slot]);        // drawer.draw + grayscale + ring.add
  e.next_slot = (e.next_slot + 1) % kSlots;
  *reward = (float)(e.mech.score - prev);
  *done = e.mech.finished;
}

void env_state_tensor(const Env& e, uint8_t* out) {
  for (int x = 0; x < kFrame; ++x)
    for (int y = 0; y < kFrame; ++y)
      for (int s = 0; s < kSlots; ++s) out[(x * kFrame + y) * kSlots + s] = e.frames[s][y * kFrame + x];
}

}  // namespace orc
