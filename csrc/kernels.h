// Host-visible argument blocks + launchers for the non-GEMM kernels.
// Every launcher is stream-ordered, allocation-free and graph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "igemm.h"

// ------------------------------------------------------------------ batch norm
struct BnApplyArgs {
  const bf16* y;
  const float* stats;            // [G][2][C]
  const float* gamma;
  const float* beta;
  const float* rmean;            // eval mode
  const float* rvar;
  int use_running;
  int res_mode;                  // 0 none, 1 identity (+res), 2 BN'd shortcut (+bn2(res))
  const bf16* res;
  const float* stats2;
  const float* gamma2;
  const float* beta2;
  const float* rmean2;
  const float* rvar2;
  bf16* out;
  int M, C, group_rows, act;     // act: 0 none, 1 relu, 2 relu6
  float eps;
};
void bn_apply_launch(const BnApplyArgs& a, hipStream_t st);
void bn_configure(long long nt_min_bytes);

struct BnBwdArgs {
  const bf16* dout;              // grad of the activation output
  const bf16* out;               // activation output (mask)
  const bf16* y;                 // conv output (pre-BN)
  const float* stats;            // [2][C]
  const float* gamma;
  const bf16* y2;                // optional shortcut conv output sharing dz
  const float* stats2;
  const float* gamma2;
  float* sums;                   // workspace [SUMS_R][3][C] (replicas, igemm.h SUMS_R)
  bf16* dy;                      // grad wrt y
  bf16* dy2;                     // grad wrt y2
  bf16* dz;                      // optional: grad wrt pre-activation (identity residual)
  float* dgamma;
  float* dbeta;
  float* dgamma2;
  float* dbeta2;
  int M, C, act;
  float eps;
  int phases;                    // 1 reduce, 2 apply, 3 both (reduce fused upstream -> 2)
};
void bn_bwd_launch(const BnBwdArgs& a, hipStream_t st);

struct BnRunEntry {
  float* rmean;
  float* rvar;
  const float* stats_train;      // [n_train][2][C]
  const float* stats_score;      // [n_score][2][C]
  long long* nbt;                // num_batches_tracked (int64) or null
  int C, n_train, n_score;
  float cnt_train, cnt_score;
};
void bn_running_launch(const BnRunEntry* tab, int nlayers, int maxC, float momentum,
                       hipStream_t st);

// ------------------------------------------------------------------ head (pool + fc + loss)
struct HeadArgs {
  const bf16* act;               // [B][HW][C] final activation
  const float* w;                // fc weight [classes][C] (fp32 master)
  const float* b;                // fc bias [classes]
  const int* label;              // [B]
  const float* isw;              // [B] importance weights N*p (train) or null (score / uniform)
  float* pooled;                 // [B][C] workspace (saved for backward)
  float* logits;                 // [B][classes] workspace
  float* dlogits;                // [B][classes] (train) or null
  float* losses;                 // [B] per-sample CE (score) or null
  float* meters;                 // [0]+=sum(w-loss)*... see head.hip
  int B, HW, C, classes, mode;   // mode 0 score, 1 train, 2 eval
  int log_softmax_input;         // logits are already log-probs (VGG) -> NLL
  int score_kind;                // losses[] holds 0: CE loss, 1: classifier-layer grad norm
  int logits_ready;              // (set by head_fwd_launch) pooled/logits already computed
  // final BatchNorm (+ identity residual) + activation applied while pooling (scoring / eval:
  // nothing else reads the last block's output): act is then the raw conv output y and
  // pooled = mean_hw(act(bn(y) [+ bn_res])) -- no bn_apply pass over the last activation
  const bf16* bn_res = nullptr;  // [B][HW][C] identity residual or null
  const float* bn_stats = nullptr;   // [G][2][C] ghost-group sums (or null: running stats)
  const float* bn_rmean = nullptr;
  const float* bn_rvar = nullptr;
  const float* bn_gamma = nullptr;   // non-null: the BN prologue is on
  const float* bn_beta = nullptr;
  float bn_inv_count = 0.f;
  float bn_eps = 0.f;
  int bn_group_imgs = 1;
  int bn_act = 0;                // 0 none, 1 relu, 2 relu6
  int pooled_ready = 0;          // (set by head_fwd_launch) pooled[] already written
};
void head_fwd_launch(const HeadArgs& a, hipStream_t st);
void head_loss_launch(const HeadArgs& a, hipStream_t st);

struct HeadBwdArgs {
  const float* pooled;           // [B][C]
  const float* dlogits;          // [B][classes]
  const float* w;                // [classes][C]
  float* dw;                     // [classes][C] fp32 grad
  float* db;                     // [classes]
  bf16* dact;                    // [B][HW][C] grad of final activation
  int B, HW, C, classes;
  // optional: also reduce the BN-backward sums of the final BN (+ shortcut BN) whose activation
  // the head read -- as a dgrad epilogue does (EpiParams bw_*): dz = dact * act'(bw_out),
  // sums[0] += dz, [1] += dz * xhat(bw_y), [2] += dz * xhat(bw_y2); [SUMS_R][3][C] replicas
  const bf16* bw_out = nullptr;
  const bf16* bw_y = nullptr;
  const float* bw_stats = nullptr;
  const bf16* bw_y2 = nullptr;
  const float* bw_stats2 = nullptr;
  float* bw_sums = nullptr;
  float bw_inv_count = 0.f, bw_eps = 0.f;
  int bw_act = 0;
};
void mlp_head_fwd_launch(const bf16* x, const bf16* w1, const float* b1, const float* w2,
                         const float* b2, float* h1, float* logits, int B, int F, int H1, int K,
                         int splits, hipStream_t st);
void mlp_head_bwd_launch(const float* dlogits, const float* h1, const bf16* x, const bf16* w1,
                         const float* w2, float* dh1, float* dw1, float* db1, float* dw2,
                         float* db2, bf16* dx, int B, int F, int H1, int K, hipStream_t st);
// returns 1 when the BN-backward sums (a.bw_sums) were reduced (the per-sample path)
int head_bwd_launch(const HeadBwdArgs& a, hipStream_t st);

// ------------------------------------------------------------------ importance sampling
struct PoolBuildArgs {
  const uint8_t* shard;          // [Ns][H][W][3] uint8 HWC
  const int64_t* labels;         // [Ns]
  const int64_t* ctrl;           // [0] pool counter (pools built so far)
  bf16* pool;                    // [P][H][W][8] bf16 normalised, channels 3..7 zero
  int* pool_label;               // [P]
  int* pool_index;               // [P] shard-local index (the dataset index the reference returns)
  int Ns, H, W, P, batch, pad, flip, augment, shuffle;
  uint32_t seed;
  float mean[3], inv_std[3];
  int prebuilt;                  // shard is already NHWC bf16 [Ns][H][W][8]: plain gather
  float* zero;                   // optional buffer zeroed by the launch (the pass's BN stats)
  int nzero;
};
void pool_build_launch(const PoolBuildArgs& a, hipStream_t st);

struct IsSampleArgs {
  const float* losses;           // [P]
  float* ema;                    // [0] value, [1] initialised flag (device-resident EMAverage)
  int64_t* ctrl;                 // [0] pool counter (incremented), [1] draw counter
  int* idx;                      // [B] drawn pool slots
  float* w;                      // [B] N * p[idx]
  float* meters;                 // [3] pool mean out, [4] ema out
  int P, B, group, importance;   // importance=0 -> uniform draws, w = 1
  float alpha, ema_alpha;
  uint32_t seed;
  int alias;                     // 1: Walker alias table in LDS + O(1) draws; 0: inverse CDF
  const float* gl;               // [W][P] all ranks' pool scores (global EMA) or null
  int W;
};
void is_sample_launch(const IsSampleArgs& a, hipStream_t st);
size_t is_sample_lds(int P, int alias);   // dynamic LDS bytes (<= 128 KB: alias up to P ~ 4k)

struct GatherArgs {
  const bf16* pool;              // [P][pix*8]
  const int* pool_label;
  const int* pool_index;
  const int* idx;                // [B]
  bf16* batch;                   // [B][pix*8]
  int* batch_label;
  int* batch_index;
  int B, chunks_per_img;         // 16-byte chunks per image
};
void gather_launch(const GatherArgs& a, hipStream_t st);

// global importance table in HBM (Groupwise sampler, K2/K11) -- csrc/table.hip
struct TableScatterArgs {
  float* imp;                    // [N] importance
  int* grp;                      // [N] group stamp
  const float* losses;           // [n]
  const int* index;              // [n] table positions, or null -> start + i
  const int64_t* stamp;          // device group id (graph-replay safe) or null -> gi
  int start, n, N, gi;
};
void table_scatter_launch(const TableScatterArgs& a, hipStream_t st);

struct TableScalars {
  float mean, count;             // group mean importance, member count
  double total;                  // sum of w = imp + mean over members
  int64_t counter;               // draw-counter snapshot used by this batch of draws
};
struct TableSampleArgs {
  const float* imp;
  const int* grp;
  int N, gi;
  const int64_t* gi_dev;         // device group id or null -> gi
  float2* part;                  // workspace [table_num_segments(N)]
  double* prefix;                // workspace [table_num_segments(N) + 1]
  TableScalars* sc;              // workspace / result scalars
  int64_t* counter;              // device draw counter (bumped once per launch) or null
  int ndraw;
  uint32_t seed;
  int64_t* out;                  // [ndraw] drawn table positions (int64) or null
  int* out32;                    // [ndraw] same as int32 or null
};
int table_num_segments(int N);
void table_sample_launch(const TableSampleArgs& a, hipStream_t st);
void table_weights_launch(const int* pos, int ndraw, const float* imp, const void* sc,
                          const int* pool_index, int Ns, int P, int* idx, float* isw,
                          float* meters, hipStream_t st);

// ------------------------------------------------------------------ optimizer
struct OptSeg {
  long long off;                 // element offset in the flat buffer (multiple of 4)
  int numel;
  int kind;                      // 0 plain, 1 conv weight (also write bf16 copies)
  int K, R, S, C, Cpad;
  bf16* w_krsc;                  // [K][R][S][Cpad] bf16 (forward / wgrad)
  bf16* w_crsk;                  // [C][R][S][K] bf16 (dgrad) or null
};
struct OptArgs {
  float* p;
  float* g;
  float* m;
  float* v;
  const OptSeg* segs;
  int nsegs;
  long long total;               // end of the swept range (padded flat length for a full step)
  const float* hyper;            // device: [0] lr [1] beta1 [2] beta2 [3] eps [4] wd
  const int64_t* step;           // device step counter (t, already incremented)
  int algo;                      // 0 adam (L2 in the gradient), 1 sgd(momentum), 2 adamw
  int zero_grad;
  long long start;               // first element of the swept range (4-aligned segment start)
};
void optimizer_launch(const OptArgs& a, hipStream_t st);
// full step in one launch: tile jobs (conv segments with a dgrad copy, C % 4 == 0) write both
// bf16 copies; ew ([n][2] start, numel) / ewp ([n+1] float4 prefix) cover everything else
void optimizer_fused_launch(const OptArgs& a, const int* jobs, int njobs, const long long* ew,
                            const long long* ewp, int new_, long long ew4, hipStream_t st);
void step_begin_launch(int64_t* ctrl, float* z0, int n0, float* z1, int n1, hipStream_t st);
// jobs: [njobs][4] = (segment index, r*S+s, k0, c0) -> one 64x64 tile each
void transpose_weights_launch(const OptSeg* segs, const int* jobs, int njobs, hipStream_t st);
void pack_weights_launch(const float* p, const OptSeg* segs, int nsegs, long long total,
                         hipStream_t st);

// ------------------------------------------------------------------ misc
void quantize_launch(const float* x, float* out, float* absmax_ws, long long n, uint32_t seed,
                     uint64_t counter, hipStream_t st);
void tern_pack_launch(const float* x, long long n, float* absmax_ws, uint32_t seed,
                      uint64_t counter, const long long* dctr, uint32_t* words, hipStream_t st);
void tern_unpack_launch(const uint32_t* msgs, int W, long long n, float scale, float* out,
                        hipStream_t st);
struct PoolArgs {                 // max-pool / avg-pool NHWC bf16
  const bf16* x;
  bf16* y;
  uint8_t* argmax;               // [N*P*Q*C] window tap r*k+s of the max, for backward, or null
  int N, H, W, C, P, Q, k, stride, pad, is_max;
  // optional BN (+ activation) of x applied per tap before pooling: x is then the raw conv
  // output, normalised from ghost-group sums ``stats`` [G][2][C] (G = N / group_imgs) or from
  // running statistics (rmean/rvar) -- the scoring pass's ImageNet stem, no bn_apply pass
  const float* stats;
  const float* gamma;
  const float* beta;
  const float* rmean;
  const float* rvar;
  int group_imgs, act;
  float eps;
};
void pool2d_fwd_launch(const PoolArgs& a, hipStream_t st);
void maxpool2d_bwd_launch(const PoolArgs& geom, const bf16* dy, bf16* dx, hipStream_t st);
struct DwArgs {                   // depthwise 3x3 conv NHWC bf16
  const bf16* x;
  const float* w;                // [C][3][3] fp32 master
  bf16* y;
  float* stats;                  // BN sums [G][2][C] or null
  int N, H, W, C, P, Q, stride, pad, group_rows;
  // input prologue (pro_gamma != null): x is the producer's raw output, act(bn(x)) is applied
  // to every loaded input chunk (padding stays zero); keep (optional) receives the activation,
  // each element written once by the thread whose strip owns it
  const float* pro_stats;        // [G][2][C] producer sums, or null -> running statistics
  const float* pro_rmean;
  const float* pro_rvar;
  const float* pro_gamma;
  const float* pro_beta;
  bf16* keep;
  float pro_inv_count, pro_eps;
  int pro_act, pro_group_imgs;
};
void dwconv_fwd_launch(const DwArgs& a, hipStream_t st);
struct StemArgs {                 // first conv: <= 4 input channels packed densely into k (stem.hip)
  const bf16* x;                  // [N][H][W][8] (channels >= C zero)
  const bf16* w;                  // [K][R][R][8] bf16 weights (channels >= C zero)
  const float* bias;              // [K] or null
  bf16* y;                        // [N][P][Q][K]
  float* stats;                   // BN sums [G][2][K] or null
  int N, H, W, K, R, stride, pad, P, Q, group_imgs;
  int tpb, blocks_per_img;        // set by the launcher
};
int stem_fwd_launch(StemArgs a, hipStream_t st);
struct DwBw {                      // BN-backward reduce fused into the depthwise dgrad
  const bf16* out;                 // activation act(bn(y)) of the BN feeding the dw conv (mask)
  const bf16* y;                   // that BN's input
  const float* stats;              // its batch sums [2][C]
  float* sums;                     // += (sum dz, sum dz * xhat) [SUMS_R][3][C] (zeroed)
  float inv_count, eps;
  int act;
};
// The dw conv's OUTPUT BatchNorm backward applied to dy as it is loaded (no bn_bwd_apply pass,
// no materialised dy): dy = A * dz + B * y + Cc per channel, dz = dout * act'(out), with
//   A = gamma * rstd, B = -A * rstd * mean(dz*xhat), Cc = A * (rstd * mean * mean(dz*xhat) -
//   mean(dz)) -- bn.hip bn_bwd_apply's arithmetic rearranged; the sums come complete from the
// producing dgrad's epilogue.  Block 0 writes that BN's dgamma / dbeta.
void dwconv_dgrad_launch(const bf16* dy, const float* w, bf16* dx, int N, int H, int W, int C,
                         int P, int Q, int stride, int pad, hipStream_t st,
                         const DwBw* bw = nullptr);
// slab (optional, >= dwconv_wgrad_slab_floats): per-block partials + a reduce kernel
size_t dwconv_wgrad_slab_floats(int N, int P, int Q, int C);
// dgrad (+ fused BN-backward sums bw) and slab wgrad of a depthwise conv in one launch; the
// partials reduce follows unless ``reduce`` is false (then dwconv_wgrad_reduce_batch_launch
// sums this layer's slab later, e.g. once for every layer at the end of the backward)
constexpr int DW_RED_MAX = 24;
int dwconv_wgrad_blocks(int N, int P, int Q, int C);
void dwconv_bwd_launch(const bf16* dy, const bf16* x, const float* w, bf16* dx, float* dw, int N,
                       int H, int W, int C, int P, int Q, int stride, int pad, float* slab,
                       const DwBw* bw, bool reduce, hipStream_t st);
void dwconv_wgrad_reduce_batch_launch(const float* const* slabs, float* const* dws, const int* Cs,
                                      const int* nblks, int n, hipStream_t st);
void dwconv_wgrad_launch(const bf16* dy, const bf16* x, float* dw, int N, int H, int W, int C,
                         int P, int Q, int stride, int pad, hipStream_t st, float* slab = nullptr,
                         size_t slab_floats = 0);
void nchw_to_nhwc8_launch(const float* x, bf16* y, int N, int C, int H, int W, int Cpad,
                          hipStream_t st);
