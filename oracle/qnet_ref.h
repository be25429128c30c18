// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h header).
//
// fp32 restatement of the reference Q-network and its train step:
//   /root/reference/src/ql-with-tensorflow/python_model/create_ql_model_breakout_84x84x4_3_32.py:20-33
//     Conv2D(32,8,s4,relu) -> Conv2D(64,4,s2,relu) -> Conv2D(64,3,s1,relu) -> Flatten -> Dense(512,relu)
//     -> Dense(3,linear); 'valid' padding, NHWC input [x][y][slot], HWIO kernels, GlorotUniform / zeros.
//   train: intended semantics q_a = Q(s)[a] (ballgame .py:71-78; the breakout .py:65-73 broadcasting bug
//     is documented, not reproduced), Keras Huber(delta=1) mean over the batch,
//     legacy Keras Adam(lr 2.5e-4, clipnorm 1.0) = tf.clip_by_norm per variable + ResourceApplyAdam
//     (op names confirmed in saved/ql_model_breakout_84x84x4_3_32/saved_model.pb).
//   batch_predict_max_future_reward = reduce_max over actions (.py:48-55); predict_action = argmax (.py:36-43).
// Accumulation is in fp32 per output element except dot products, which accumulate in double
// (a tighter reference than TF's unknown reduction order; the product's tolerance is stated
// against this oracle in tests/).
#pragma once
#include <cstdint>
#include <vector>

namespace orc {

constexpr int kNumVars = 10;
constexpr int kActions = 3;

struct VarShape { int rows, cols; };   // flattened [fan-in dims..., out]
// k0 [8,8,4,32] b0 [32] k1 [4,4,32,64] b1 [64] k2 [3,3,64,64] b2 [64] k3 [3136,512] b3 [512] k4 [512,3] b4 [3]
extern const int kVarSize[kNumVars];

struct QNet {
  std::vector<float> w[kNumVars];
  std::vector<float> m[kNumVars];
  std::vector<float> v[kNumVars];
  int64_t iterations = 0;
  float lr = 0.00025f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-7f, clipnorm = 1.0f;
};

void qnet_init_glorot(QNet& q, uint64_t seed);
void qnet_copy_weights(QNet& dst, const QNet& src);

struct Acts {   // activations kept for backward (post-ReLU)
  std::vector<float> a1, a2, a3, a4, q;   // [B,20,20,32] [B,9,9,64] [B,7,7,64] [B,512] [B,3]
};

// x: u8 [B][84][84][4] (reference tensor view, exact in f32)
void qnet_forward(const QNet& q, const uint8_t* x, int B, Acts& acts);

struct Grads { std::vector<float> g[kNumVars]; };
// Huber loss + full backward. Returns the loss; grads are the raw (unclipped) gradients.
// weights (optional): per-sample loss weights (prioritized-replay IS weights); td_abs (optional): |q_a - y| out
float qnet_loss_backward(const QNet& q, const uint8_t* x, const uint8_t* actions, const float* y, int B,
                         const Acts& acts, Grads& grads, const float* weights = nullptr, float* td_abs = nullptr);
// clip_by_norm per variable + ResourceApplyAdam, iterations += 1
void qnet_apply_adam(QNet& q, const Grads& grads, float* norms_out /*[10] or null*/);

// The fp32 arithmetic of the product's QLX_ARCH_NATURE_DQN (qnet32_ref.cpp): the same math with every reduction a
// single fmaf chain in the order the build defines, so the GPU results match bit for bit.
void qnet32_forward(const QNet& q, const uint8_t* x, int B, Acts& acts);
float qnet32_loss_backward(const QNet& q, const uint8_t* x, const uint8_t* actions, const float* y, int B,
                           const Acts& acts, Grads& grads, const float* weights = nullptr, float* td_abs = nullptr);
void qnet32_apply_adam(QNet& q, const Grads& grads, float* norms_out /*[10] or null*/);
// the product's dense-frame path (QLX_F32_BG=0): the conv weight gradients over every row (no background-row
// compaction); process-wide, default off
void qnet32_set_dense(bool dense);

// reference helpers
int argmax_first(const float* q, int n);

}  // namespace orc
