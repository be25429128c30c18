// Host-side Q-network object and the launch helpers the learner composes.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "profiler.h"
#include "qlx_internal.h"

namespace qlx {

constexpr int kNumVars = 10;
constexpr int64_t kVarOffsetDense = 77984;   // flat offset of W3 (conv variables before it, dense ones after)
constexpr int64_t kNumParams = 1685667;   // sum of the 10 Keras variables (variables.index shapes)
constexpr int kFc1Split = 4;              // bf16: split-K of the 3136-deep dense layer at training batches (25 / 23 k-steps)
// conv weight-gradient partial slabs, one region per layer (conv3 and conv2 share a launch)
constexpr size_t kSlabConv3 = 0, kSlabConv2 = (size_t)3200 * 1024, kSlabConv1 = (size_t)7424 * 1024;
constexpr size_t kWgradSlabFloats = (size_t)9600 * 1024;
constexpr size_t kBiasSlabFloats = 256 * 512;
extern const int kVarSize[kNumVars];

struct ModelWs {   // per-batch workspace (activations are bf16, heads fp32)
  uint8_t* frames = nullptr;          // [B*4][7056] s2d staging for host observations
  const uint8_t** table = nullptr;    // [B][4] frame pointers
  __bf16 *a1 = nullptr, *a2 = nullptr, *a3 = nullptr, *a4 = nullptr;
  __bf16 *dz1 = nullptr, *dz2 = nullptr, *dz3 = nullptr, *dz4 = nullptr;
  float* q = nullptr;
  float *gs = nullptr, *hs = nullptr, *y = nullptr, *rew = nullptr;
  uint8_t *act = nullptr, *argmax = nullptr, *done = nullptr;
  float* fc1slab = nullptr;
  int a4_splits = 0;                  // > 0: a4 still pending as that many split-K fc1 partials in fc1slab
  float* slab = nullptr;
  float* bslab = nullptr;
  float* loss = nullptr;
  // fp32 path (qnet32.hip): activations a1..a3 per forward chunk of `fchunk` samples, a4 for the whole batch; the
  // gradient buffers (dz, weight-gradient chunk slabs) in their own allocation `fgrad`, sized for fgrad_batch
  float *fa1 = nullptr, *fa2 = nullptr, *fa3 = nullptr, *fa4 = nullptr;
  float *fdz1 = nullptr, *fdz2 = nullptr, *fdz3 = nullptr, *fdz4 = nullptr;
  float *fslab1 = nullptr, *fslab2 = nullptr, *fslab3 = nullptr;
  float* fpb1 = nullptr;    // conv1 bias partials of the conv2 backward [ceil(B / 16)][400][32]
  float* fpbg2 = nullptr;   // conv2 background-row dz2 partials of the conv3 backward [ceil(B / 16)][81][64]
  float* fs2 = nullptr;     // their per-chunk sums [ceil(B / 16)][64] (SideBgSum)
  float* fpbg3 = nullptr;   // conv3 background-row dz3 partials of the fc1 backward [ceil(B / 16)][49][64]
  float* fs3 = nullptr;     // their per-chunk sums [ceil(B / 16)][64]
  float* fpart = nullptr;   // clip_by_norm segment partials
  // background rows of the conv2 / conv3 forward (qnet32_kernels.h C1Lists): row lists of the forward chunk, the list
  // counters of two forwards (double-buffered by forward parity), the constant rows relu(b0) / c2 / c3
  int *frl2 = nullptr, *frl3 = nullptr;
  unsigned long long* frcnt = nullptr;
  float* fbgc = nullptr;
  uint32_t* fsteps = nullptr;   // the forward chunk's conv1 step masks [fchunk][4] (written when the row lists are)
  uint8_t* fneed = nullptr;     // the same bits as bytes [100][fneed_ld] (step-major)
  int fneed_ld = 0;
  uint32_t* frows2 = nullptr;   // the forward chunk's conv2 non-background row bits [fchunk][4]
  uint8_t* fbg2 = nullptr;      // its conv2 background rows as bytes [81][fneed_ld]
  uint32_t* frows3 = nullptr;   // the same for conv3 [fchunk][4], [49][fneed_ld]
  uint8_t* fbg3 = nullptr;
  int fparity = 0;
  int frl_cap = 0;   // samples the row lists hold
  int fchunk = 0;
  void* fgrad = nullptr;
  int fgrad_batch = 0;
};

constexpr int kF32FwdChunk = 8192;   // samples per fp32 forward pass (bounds the a1..a3 workspace)

}  // namespace qlx

struct qlx_model {
  int device = 0;
  bool f32 = true;   // QLX_ARCH_NATURE_DQN: fp32 (the reference's arithmetic); QLX_ARCH_NATURE_DQN_BF16: bf16 MFMA operands
  hipStream_t stream = nullptr;
  bool own_stream = true;
  float* d_params = nullptr;   // fp32 master weights, Keras layouts, variables concatenated
  float* d_m = nullptr;
  float* d_v = nullptr;
  float* d_grads = nullptr;
  // bf16 MFMA operand copies ([n][k], k contiguous)
  __bf16 *wf0 = nullptr, *wf1 = nullptr, *wb1 = nullptr, *wf2 = nullptr, *wb2 = nullptr, *wb3 = nullptr;
  int64_t iterations = 0;
  uint64_t version = 0;   // bumped by model_pack, i.e. on every write of the weights from outside the optimizer
  float lr = 0.00025f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-7f, clipnorm = 1.0f;
  int n_ranges = 0;
  int64_t *d_rbeg = nullptr, *d_rend = nullptr;
  float* d_partial = nullptr;
  int* d_var_first = nullptr;
  // clip_by_norm partials written by the gradient producers themselves (fc1 wgrad tiles, conv slab reduction
  // blocks, fc2 wgrad blocks): when no all-reduce sits between backward and Adam the k_sumsq pass is skipped
  float* d_sqf = nullptr;
  int* d_sqf_first = nullptr;
  bool norms_fused = false;   // set by model_norms: Adam reads d_sqf / d_sqf_first instead
  float* d_norms = nullptr;
  // XCD-aware block -> tile table of the fc1 backward launch (built per batch size, qnet.hip fc1_bwd_map)
  int* d_fc1bwd_map = nullptr;
  int fc1bwd_map_B = -1, fc1bwd_grid = 0, fc1bwd_cap = 0;
  void* ws = nullptr;
  int ws_batch = 0;
  int last_batch = 0;
  qlx::ModelWs w;
  qlx::Profiler* prof = nullptr;   // set by the learner while profiling
  // conv1 weight gradient as channel-half blocks (k_conv1_wgrad_h); QLX_CONV1_HALVES=0 at create time selects the
  // one-block-per-chunk k_conv1_wgrad (bit-identical gradients)
  bool conv1_halves = true;
  // fp32 sparsity paths, read at create time (a learner built with them off runs the dense forward / weight gradient in
  // the same process: bench.py value_dense_frames): QLX_F32_BG=0 computes every conv2 / conv3 forward row (no background
  // rows), QLX_F32_C1_SKIP=0 issues conv1's all-zero frame steps.  Bit-identical results either way.
  bool f32_bg_rows = true;
  int f32_c1_skip = 1;
  // fp32 update schedule (when the caller allows it: no all-reduce between backward and Adam): the dense variables' norm
  // partials as extra blocks of the weight-gradient reduction launch, then every variable's clip_by_norm + Adam in one
  // launch (k_update32) - the update's tail is two launches.  Set by the backward, consumed by model_norms / model_adam.
  bool f32_update_scheduled = false;
  // data parallel (an all-reduce between the backward and the update): model_norms wrote the dense variables' norm
  // partials of the reduced gradient x f32_partials_scale; model_adam then runs the same k_update32 tail
  bool f32_dense_partials = false;
  float f32_partials_scale = 1.0f;
  // dense-variable update beside the conv backward (QLX_F32_DENSE_OVERLAP, scheduled update only): the dense clip-norm
  // partials + Adam run on f32_aux from the end of the fc1 backward; the next fc1 forward (and every host-visible sync of
  // the model) joins it.  f32_dense_async: this update's dense part went to f32_aux (k_update32 then runs the conv blocks).
  bool dense_overlap = false;
  bool f32_dense_async = false;
  bool dense_pending = false;
  hipStream_t f32_aux = nullptr;
  hipEvent_t ev_dense_ready = nullptr, ev_dense_done = nullptr;
  // bf16 forward: fc1 as one pass with the fused epilogue at every batch size (no batch-size-dependent split-K), so a
  // sample's result does not depend on the batch it is evaluated in (the learner's target net)
  bool fc1_single = false;
};

namespace qlx {
struct Fc2Args {
  const __bf16* a4;          // [B][512]
  const float* a4f;          // fp32 model: [B][512]
  // pending split-K fc1 partials (splits > 0): the head finishes a4 = relu(sum_z slab[z] + b3) in fixed z order
  // and writes it to a4_out, so no separate reduction launch runs
  const float* slab;
  size_t zstride;
  int splits;
  const float* b3;
  __bf16* a4_out;
  const float* w4;         // [512][3] master
  const float* b4;         // [3]
  int B;
  float* q;                // [B][3] out (may be null)
  uint8_t* argmax;         // mode 1
  const float* rewards;    // mode 2
  const uint8_t* dones;    // mode 2
  float gamma;             // mode 2
  float* y_out;            // mode 2
  const float* q_select;   // mode 2, double DQN: [B][3] online Q(s'), a* = its first argmax, y uses q[a*] (else max)
  const uint8_t* actions;  // training head
  const float* y;          // training head
  float* gsample;          // training head: dloss/dq_a per sample
  float* hsample;          // training head: per-sample Huber value
  const float* weights;    // training head (optional): per-sample loss weights (prioritized-replay IS weights)
  float* td_abs;           // training head (optional): |q_a - y| out
  float* dz4_out;          // fp32 training head (optional): the dense-3 backward dz4 [B][512], fused
};
// fc2 kernel arguments for the model's last forward; consumes pending fc1 partials (the fc2 launch that
// follows materialises a4)
Fc2Args fc2_args(qlx_model* m, int B);
void launch_fc2(int mode, const Fc2Args& a, int B, hipStream_t s);
void model_workspace(qlx_model* m, int B);
void model_pack(qlx_model* m);
// store_acts = false skips writing a1/a2 (only a3 is needed when no backward pass follows)
void model_forward_trunk(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s, bool store_acts = true);
// Huber head + backward after model_forward_trunk: loss -> *loss_dev, raw gradients -> m->d_grads
// weights (optional): per-sample loss weights; td_abs (optional): |q_a - y| per sample out.
// = model_backward_dense (head, fc1: the dense gradients, 95 % of the bytes, are final after it) followed by
// model_backward_conv (the conv trunk); a data-parallel caller all-reduces the dense bucket in between
// fuse_update: no all-reduce will follow, so the fp32 path may schedule the norms / Adam of the variables whose gradient
// is final inside the later backward launches (model_norms / model_adam then finish the rest)
void model_backward(qlx_model* m, const uint8_t* const* table, int B, const uint8_t* actions, const float* y, float* loss_dev,
                    hipStream_t s, const float* weights = nullptr, float* td_abs = nullptr, bool fuse_update = false);
void model_backward_dense(qlx_model* m, int B, const uint8_t* actions, const float* y, float* loss_dev, hipStream_t s,
                          const float* weights = nullptr, float* td_abs = nullptr);
// dense_ready (fp32, data parallel): the dense bucket's all-reduce event; the reduction launch then waits for it and computes
// the dense variables' clip-norm partials of the reduced gradient x dense_scale as its extra blocks (no f32_norms launch)
void model_backward_conv(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s, bool fuse_update = false,
                         hipEvent_t dense_ready = nullptr, float dense_scale = 1.0f);
// per-variable norm partials for Adam: with scale == 1 (no all-reduce since the backward) the producers'
// fused partials are used as they are; otherwise per-range sums of squares of the scaled gradients
void model_norms(qlx_model* m, hipStream_t s, float scale);
void model_adam(qlx_model* m, hipStream_t s, float scale);

// fp32 path (qnet32.hip), dispatched to by the model_* functions when m->f32
void f32_workspace(qlx_model* m, int B);
void f32_forward(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s);
void f32_head(int mode, const Fc2Args& a, int B, hipStream_t s);   // mode 3 = training head
void f32_backward_dense(qlx_model* m, int B, const uint8_t* actions, const float* y, float* loss_dev, hipStream_t s,
                        const float* weights, float* td_abs);
void f32_backward_conv(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s, bool fuse_update,
                       hipEvent_t dense_ready = nullptr, float dense_scale = 1.0f);
void f32_norms(qlx_model* m, hipStream_t s, float scale);
void f32_adam(qlx_model* m, hipStream_t s, float scale);
// the dense variables' norm partials + Adam of the update in flight on m->f32_aux (after the fc1 backward on s)
void f32_dense_async(qlx_model* m, hipStream_t s);
// stream s waits for a pending dense update (before anything reads W3 / b3 / W4 / b4 again)
void model_dense_join(qlx_model* m, hipStream_t s);
// fractions of a batch's fp32 conv work the exact skips leave out (qnet32.hip k_frame_sparsity; synchronises s):
// out = {conv1 forward zero steps, conv1 weight-gradient zero steps, conv2 background rows, conv3 background rows}
// d_cnt: 4 device counters, h_cnt: their pinned host copy (both the caller's, allocated once)
void frame_sparsity(const uint8_t* const* table, int n, unsigned long long* d_cnt, unsigned long long* h_cnt, double* out,
                    hipStream_t s);
}  // namespace qlx
