// Classifier head: global average pool + linear + (importance-weighted) cross-entropy.
//
// Score mode is the reference's presample loss (`pytorch_collab.py:101-102`,
// `F.cross_entropy(reduction='none')`): per-sample
// l_i = logsumexp(z_i) - z_i[y_i].  Train mode is K4: the IS-weighted loss
// mean_i(l_i / w_i) (`:133-145`) and its gradient
// dz_i = (softmax(z_i) - onehot(y_i)) / (B * w_i), written in the same launch,
// plus device-side meters (loss sum, sample count, correct count) so the hot
// loop never syncs for `.item()` (`util.py:226-231`).
//
// One workgroup per sample: the pooled feature vector and the logits stay in
// LDS; dot products are wave64 reductions.
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

__global__ __launch_bounds__(NT) void head_fwd_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* pooled = sh;               // [C]
  float* logit = sh + a.C;          // [classes]
  float* red = logit + a.classes;   // [16]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bf16* x = a.act + (size_t)b * a.HW * a.C;
  const float invhw = 1.f / (float)a.HW;
  for (int c = tid; c < a.C; c += NT) {
    float s = 0.f;
#pragma unroll 8
    for (int hw = 0; hw < a.HW; ++hw) s += bf2f(x[(size_t)hw * a.C + c]);
    s *= invhw;
    pooled[c] = s;
    if (a.pooled) a.pooled[(size_t)b * a.C + c] = s;
  }
  __syncthreads();
  for (int k = wv; k < a.classes; k += NT / 64) {
    const float* wr = a.w + (size_t)k * a.C;
    float d = 0.f;
#pragma unroll 8
    for (int c = lane; c < a.C; c += 64) d += wr[c] * pooled[c];
    d = wave_sum(d);
    if (lane == 0) logit[k] = d + (a.b ? a.b[k] : 0.f);
  }
  __syncthreads();
  // log-sum-exp and argmax, one wave
  if (wv == 0) {
    float mx = -3.4e38f;
    int am = 0;
    for (int k = lane; k < a.classes; k += 64) {
      if (logit[k] > mx) {
        mx = logit[k];
        am = k;
      }
    }
    // wave argmax (first max wins on ties, like torch.argmax)
    for (int o = 32; o >= 1; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oa < am)) {
        mx = om;
        am = oa;
      }
    }
    float se = 0.f;
    for (int k = lane; k < a.classes; k += 64) se += __expf(logit[k] - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    const int y = a.label[b];
    const float loss = lse - logit[y];
    float score = loss;
    if (a.score_kind == 1) {
      // exact per-sample gradient norm of the classifier layer: d(loss)/d[W|b] is the outer
      // product of dz = softmax - onehot with [h, 1], so its Frobenius norm factorises
      float g2 = 0.f, h2 = 0.f;
      for (int k = lane; k < a.classes; k += 64) {
        const float d = __expf(logit[k] - lse) - (k == y ? 1.f : 0.f);
        g2 += d * d;
      }
      for (int c = lane; c < a.C; c += 64) h2 += pooled[c] * pooled[c];
      score = sqrtf(wave_sum(g2) * (wave_sum(h2) + 1.f));
    }
    if (lane == 0) {
      if (a.losses) a.losses[b] = score;
      red[0] = lse;
      const float wi = a.isw ? a.isw[b] : 1.f;
      if (a.mode == 1 || a.mode == 2) {
        if (a.meters) {
          atomicAdd(&a.meters[0], a.mode == 1 ? loss / wi : loss);
          atomicAdd(&a.meters[1], 1.f);
          atomicAdd(&a.meters[2], am == y ? 1.f : 0.f);
        }
      }
      red[1] = 1.f / ((float)a.B * wi);
    }
  }
  __syncthreads();
  if (a.mode == 1 && a.dlogits) {
    const float lse = red[0], scale = red[1];
    const int y = a.label[b];
    for (int k = tid; k < a.classes; k += NT) {
      const float p = __expf(logit[k] - lse);
      a.dlogits[(size_t)b * a.classes + k] = (p - (k == y ? 1.f : 0.f)) * scale;
    }
  }
}

// grid = (channel blocks, B + classes): block row y < B writes sample y's activation
// gradient (d pooled / HW broadcast over the spatial positions); row B + k reduces
// dW[k][:] (and db[k]) over the batch.  Every thread's loop is short and unrolled so
// its loads are in flight together.
__global__ __launch_bounds__(NT) void head_bwd_kernel(HeadBwdArgs a) {
  const int c = blockIdx.x * NT + threadIdx.x;
  const int b = blockIdx.y;
  if (b >= a.B) {
    const int k = b - a.B;
    if (blockIdx.x == 0 && threadIdx.x < 64) {
      float s = 0.f;
      for (int i = threadIdx.x; i < a.B; i += 64) s += a.dlogits[(size_t)i * a.classes + k];
      s = wave_sum(s);
      if (threadIdx.x == 0) a.db[k] = s;
    }
    if (c >= a.C) return;
    float s = 0.f;
#pragma unroll 8
    for (int i = 0; i < a.B; ++i)
      s += a.dlogits[(size_t)i * a.classes + k] * a.pooled[(size_t)i * a.C + c];
    a.dw[(size_t)k * a.C + c] = s;
    return;
  }
  if (c >= a.C) return;
  float s = 0.f;
#pragma unroll 8
  for (int k = 0; k < a.classes; ++k)
    s += a.dlogits[(size_t)b * a.classes + k] * a.w[(size_t)k * a.C + c];
  const bf16 v = f2bf(s / (float)a.HW);
  bf16* dst = a.dact + (size_t)b * a.HW * a.C + c;
  for (int hw = 0; hw < a.HW; ++hw) dst[(size_t)hw * a.C] = v;
}
}  // namespace

void head_fwd_launch(const HeadArgs& a, hipStream_t st) {
  const size_t shm = (size_t)(a.C + a.classes + 16) * sizeof(float);
  hipLaunchKernelGGL(head_fwd_kernel, dim3(a.B), dim3(NT), shm, st, a);
}

void head_bwd_launch(const HeadBwdArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(head_bwd_kernel, dim3((a.C + NT - 1) / NT, a.B + a.classes), dim3(NT), 0, st,
                     a);
}
