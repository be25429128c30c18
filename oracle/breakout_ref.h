// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h header).
//
// CPU restatement of the reference's Breakout physics and environment:
//   /root/reference/src/breakout-game/src/mechanics.rs      (all of it)
//   /root/reference/src/breakout-game/src/algebra_2d.rs     (reflect / angle / contact)
//   /root/reference/src/_breakout-ml/src/breakout_environment.rs:15,39-77,94-120,155-161,173-207
//   /root/reference/src/_breakout-ml/src/util/frame_ring_buffer.rs:17-63
// Third-party arithmetic restated from published sources (not vendored in the reference):
//   emath 0.22 Vec2 (length = f32::hypot, normalized = v / len unless len <= 0),
//   parry2d 0.13.8 query::contact(Ball, Cuboid) = contact_ball_convex_polyhedron
//     (AABB point projection + Unit::try_new_and_get, prediction 0.8),
//   glibc 2.35 hypotf / acosf (Rust std's f32::hypot / f32::acos call libm).
// Compiled with -ffp-contract=off: Rust never fuses a*b+c.
#pragma once
#include <cstdint>
#include <vector>

namespace orc {

struct V2 { float x, y; };
struct AABB { V2 min, max; };

struct ContactSurface {   // algebra_2d.rs:37-43
  float way;
  float approximation;
  V2 normal;
};

struct Brick { AABB shape; int id; };   // id = creation order 0..59 (rows top→bottom, left→right)

struct Mechanics {   // mechanics.rs:46-54
  std::vector<Brick> bricks;
  V2 ball_center;
  float ball_radius;
  V2 ball_dir;
  float ball_speed;
  AABB panel;
  float panel_speed;
  bool finished;
  uint32_t score;
  int fault;          // non-zero where the reference would panic (assert!) — see fault codes
};

enum Fault : int {
  F_OK = 0,
  F_WALL_ASSERT = 1,       // mechanics.rs:265/284/303 assert!(wall_distance >= 0)
  F_CANDIDATE_ASSERT = 2,  // mechanics.rs:511 assert!(approximation in range)
  F_RECURSION = 4,         // bounded stand-in for the reference's unbounded recursion
};

constexpr int kFrame = 84;
constexpr int kFramePix = kFrame * kFrame;   // 7056
constexpr int kSlots = 4;                    // breakout_environment.rs:15
constexpr int kNumBricks = 60;

// Build-defined rasterizer palette (reference drawer is unimplemented!(): breakout_drawer.rs:22-28).
// Colours from app_game_drawer.rs:55-86 converted with image 0.24 rgb_to_luma
// ((2126 r + 7152 g + 722 b) / 10000, integer): DARK_GRAY(96,96,96)=96, YELLOW(255,255,0)=236,
// WHITE=255, background BLACK=0.
constexpr uint8_t kLumaBrick = 96, kLumaBall = 236, kLumaPanel = 255;

void mechanics_init(Mechanics& m, uint64_t seed, uint32_t env_id, uint32_t reset_count);
void mechanics_time_step(Mechanics& m, int action);   // action 0 None, 1 Left, 2 Right
float acos_gt_half_pi_threshold();                    // see breakout_ref.cpp

// KAT entry points (mechanics.rs:659-752)
bool wall_left(V2 center, float radius, V2 mv, ContactSurface* out, int* fault);
bool wall_right(V2 center, float radius, V2 mv, ContactSurface* out, int* fault);
bool rect_check(V2 center, float radius, V2 mv, AABB rect, ContactSurface* out);

// Rasterize the mechanics into an 84x84 grayscale image, row-major [y][x] (ImageBuffer order).
void rasterize(const Mechanics& m, uint8_t* img_yx);

struct Env {   // BreakoutEnvironment + BreakoutState
  Mechanics mech;
  uint8_t frames[kSlots][kFramePix];   // FrameRingBuffer.buffer, each [y][x]
  int next_slot;
  uint64_t seed;
  uint32_t env_id;
  uint32_t reset_count;
};

void env_init(Env& e, uint64_t seed, uint32_t env_id);
void env_reset(Env& e);                                   // breakout_environment.rs:177-180
void env_step(Env& e, int action, float* reward, bool* done);   // :184-201
// ToMultiDimArray view: tensor[x][y][slot] (breakout_environment.rs:44-50), 28,224 bytes.
void env_state_tensor(const Env& e, uint8_t* out_xys);

}  // namespace orc
