// Direct-xGMI two-shot all-reduce: the GPU counterpart of the reference's
// hand-written CPU ring (`util.py:280-324`), designed for MI355X's fully connected xGMI
// (7 point-to-point links per GPU, ~153 GB/s each) instead of a ring.
//
// A ring all-reduce moves every byte over ONE link per step, so on an 8-GPU node it uses 2 of
// the 7 links of each GPU.  Here every rank has an exchange buffer that every peer maps with
// hipIpcOpenMemHandle, and the reduction is two direct passes:
//
//   reduce-scatter : rank r owns chunk r (n / W elements, 16-byte aligned); one kernel reads
//                    chunk r from ALL W exchange buffers at once (W-1 of them remote: all 7
//                    links busy in parallel), sums in fp32 and writes the result into chunk r
//                    of its own exchange buffer;
//   all-gather     : one kernel reads chunk p of peer p's exchange buffer for every p and
//                    writes the full reduced vector into the local destination.
//
// Each rank moves 2 (W-1)/W n elements over xGMI -- the same as a ring -- but spread over
// W-1 links instead of one.  The passes are separated by stream-ordered barriers: a one-block
// kernel that writes this rank's epoch into every peer's flag slot (system-scope atomic
// stores into the IPC-mapped flag area) and polls its own flag area until every peer has
// written the same epoch (bounded: a peer that never arrives sets an error word and the kernel
// exits instead of spinning forever).  Host barriers remain for tests.  Exchange-buffer traffic uses system-coherent (sc0|sc1)
// buffer loads and stores, so no reader depends on kernel-boundary cache maintenance.  ``wire_bf16``: the exchange buffers hold bf16 (half the
// bytes over the links); sums are accumulated in fp32 and rounded once per pass.
//
// For testing on one GPU the "peers" are simply W local buffers (emulated ranks).
#include <algorithm>
#include <string>

#include "common.h"

namespace {

constexpr int XMAX = 8;

struct Peers {
  const void* p[XMAX];
};

// Every access to an exchange buffer is SYSTEM-coherent (buffer ops with sc0|sc1): the buffers
// are ordinary coarse-grained allocations mapped into the peers over IPC, and a reader's
// non-coherent L2 could otherwise serve a line cached from the previous bucket that used the
// same address -- a failure one GPU (where all "peers" share an L2) can never show.  Stores are
// written through to memory for the same reason.  (Streaming, so the bypass costs nothing.)
constexpr int SYS = 1 | 16;   // sc0 | sc1

typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;

MA_DEV __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000);
}

MA_DEV f32x4 ld4(__amdgpu_buffer_rsrc_t r, long long i, bool bf) {
  if (!bf) return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, SYS));
  // bf16 -> f32 by integer shifts (bf16x2 bit-casts of the loaded dwords miscompiled: hipcc
  // dropped the second dword and loaded 4 bytes)
  const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(i * 8), 0, SYS);
  return f32x4{__uint_as_float(v[0] << 16), __uint_as_float(v[0] & 0xffff0000u),
               __uint_as_float(v[1] << 16), __uint_as_float(v[1] & 0xffff0000u)};
}

MA_DEV unsigned bf16_bits(float x) { return (unsigned)__builtin_bit_cast(unsigned short, f2bf(x)); }

MA_DEV void st4(__amdgpu_buffer_rsrc_t r, long long i, f32x4 v, bool bf) {
  if (!bf) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)(i * 16), 0, SYS);
    return;
  }
  const u32x2_t o{bf16_bits(v[0]) | (bf16_bits(v[1]) << 16), bf16_bits(v[2]) | (bf16_bits(v[3]) << 16)};
  __builtin_amdgcn_raw_buffer_store_b64(o, r, (int)(i * 8), 0, SYS);
}

// chunk r = [off(r), off(r+1)) in float4 units
__host__ __device__ inline long long chunk_off(long long n4, int W, int r) { return r >= W ? n4 : n4 * r / W; }

template <bool BF>
__global__ __launch_bounds__(256) void xgmi_rs_kernel(Peers peers, int W, int rank, long long n4,
                                                      float scale) {
  const long long bytes = n4 * (BF ? 8 : 16);
  __amdgpu_buffer_rsrc_t r[XMAX];
#pragma unroll
  for (int q = 0; q < XMAX; ++q) r[q] = rsrc(peers.p[q < W ? q : 0], bytes);
  const long long c0 = chunk_off(n4, W, rank), c1 = chunk_off(n4, W, rank + 1);
  for (long long i = c0 + (long long)blockIdx.x * 256 + threadIdx.x; i < c1;
       i += (long long)gridDim.x * 256) {
    f32x4 acc = ld4(r[0], i, BF);
#pragma unroll
    for (int q = 1; q < XMAX; ++q)
      if (q < W) acc += ld4(r[q], i, BF);
    st4(r[rank < XMAX ? rank : 0], i, acc * scale, BF);
  }
}

// dst (fp32, local) <- chunk p of peer p: blockIdx.y = p, one contiguous stream per peer (all
// W-1 remote links read in parallel, no per-element owner search)
template <bool BF>
__global__ __launch_bounds__(256) void xgmi_ag_kernel(Peers peers, int W, long long n4,
                                                      float* __restrict__ dst) {
  const int p = blockIdx.y;
  const auto r = rsrc(peers.p[p], n4 * (BF ? 8 : 16));
  const long long c0 = chunk_off(n4, W, p), c1 = chunk_off(n4, W, p + 1);
  for (long long i = c0 + (long long)blockIdx.x * 256 + threadIdx.x; i < c1;
       i += (long long)gridDim.x * 256)
    ((f32x4*)dst)[i] = ld4(r, i, BF);
}

template <bool BF>
__global__ __launch_bounds__(256) void xgmi_pack_kernel(const float* __restrict__ src,
                                                        void* __restrict__ xbuf, long long n4) {
  const auto r = rsrc(xbuf, n4 * (BF ? 8 : 16));
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (long long)gridDim.x * 256)
    st4(r, i, ((const f32x4*)src)[i], BF);
}

unsigned grid_for(long long n4) {
  long long b = (n4 + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

}  // namespace

// n: element count (a multiple of 4; the engine's buckets are 4-aligned flat ranges)
void xgmi_pack(const float* src, void* xbuf, long long n, int bf, hipStream_t st) {
  const long long n4 = n / 4;
  if (bf)
    hipLaunchKernelGGL(xgmi_pack_kernel<true>, dim3(grid_for(n4)), dim3(256), 0, st, src, xbuf, n4);
  else
    hipLaunchKernelGGL(xgmi_pack_kernel<false>, dim3(grid_for(n4)), dim3(256), 0, st, src, xbuf, n4);
}

void xgmi_reduce_scatter(const void* const* peers, int W, int rank, long long n, int bf,
                         float scale, hipStream_t st) {
  Peers p{};
  for (int q = 0; q < W && q < XMAX; ++q) p.p[q] = peers[q];
  const long long n4 = n / 4;
  const long long mine = chunk_off(n4, W, rank + 1) - chunk_off(n4, W, rank);
  if (bf)
    hipLaunchKernelGGL(xgmi_rs_kernel<true>, dim3(grid_for(mine)), dim3(256), 0, st, p, W, rank,
                       n4, scale);
  else
    hipLaunchKernelGGL(xgmi_rs_kernel<false>, dim3(grid_for(mine)), dim3(256), 0, st, p, W, rank,
                       n4, scale);
}

void xgmi_all_gather(const void* const* peers, int W, long long n, int bf, float* dst,
                     hipStream_t st) {
  Peers p{};
  for (int q = 0; q < W && q < XMAX; ++q) p.p[q] = peers[q];
  const long long n4 = n / 4;
  const dim3 grid(grid_for((n4 + W - 1) / W), W);
  if (bf)
    hipLaunchKernelGGL(xgmi_ag_kernel<true>, grid, dim3(256), 0, st, p, W, n4, dst);
  else
    hipLaunchKernelGGL(xgmi_ag_kernel<false>, grid, dim3(256), 0, st, p, W, n4, dst);
}

// ---------------------------------------------------------------- device-side barrier
// Flag area: XMAX slots of 128 B (one line each) at the head of every rank's exchange
// allocation; slot q of rank r's area is written ONLY by rank q.  The epoch is this rank's
// count of barriers (all ranks run the same sequence, graph replays included), so a slot
// holding epoch e means that peer has reached barrier e.
constexpr int FLAG_STRIDE = 32;    // uint32 per slot (128 B)

__global__ __launch_bounds__(64) void xgmi_barrier_kernel(Peers flags, unsigned* own, int W,
                                                          int rank, unsigned* epoch,
                                                          unsigned long long timeout, int* err) {
  const int q = threadIdx.x;
  const unsigned e = epoch[0] + 1u;
  // everything this rank wrote into its exchange buffer before the barrier (earlier kernels of
  // this stream, system-coherent stores) is visible system-wide before the signal
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (q < W && q != rank) {
    unsigned* slot = (unsigned*)flags.p[q] + rank * FLAG_STRIDE;
    __hip_atomic_store(slot, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* mine = own + q * FLAG_STRIDE;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(4);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {   // 100 MHz ticks
        atomicOr(err, 1 << q);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (q == 0) epoch[0] = e;
}

int xgmi_max_ranks() { return XMAX; }

// IPC: export a device allocation / map a peer's (one process per GPU; HSA_ENABLE_IPC_MODE_LEGACY=0)
std::string xgmi_ipc_handle(uintptr_t ptr) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, (void*)ptr) != hipSuccess) return std::string();
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

uintptr_t xgmi_ipc_open(const std::string& handle) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) return 0;
  hipIpcMemHandle_t h;
  std::copy(handle.begin(), handle.end(), reinterpret_cast<char*>(&h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return 0;
  return reinterpret_cast<uintptr_t>(p);
}

void xgmi_barrier(const void* const* flag_areas, int W, int rank, unsigned* epoch,
                  double timeout_s, int* err, hipStream_t st) {
  Peers p{};
  for (int q = 0; q < W && q < XMAX; ++q) p.p[q] = flag_areas[q];
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);
  hipLaunchKernelGGL(xgmi_barrier_kernel, dim3(1), dim3(64), 0, st, p, (unsigned*)flag_areas[rank],
                     W, rank, epoch, ticks, err);
}

int xgmi_flag_bytes() { return XMAX * FLAG_STRIDE * 4; }

uintptr_t xgmi_malloc(long long bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, (size_t)bytes) != hipSuccess) return 0;
  (void)hipMemset(p, 0, (size_t)bytes);
  return reinterpret_cast<uintptr_t>(p);
}

void xgmi_free(uintptr_t p) {
  if (p) (void)hipFree(reinterpret_cast<void*>(p));
}

void xgmi_ipc_close(uintptr_t p) {
  if (p) (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(p));
}
