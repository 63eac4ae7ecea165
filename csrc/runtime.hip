// Runtime checks for the engine's multi-stream step (race detection).
//
// The native step runs on up to three HIP streams -- scoring, train (fwd/bwd + tail) and the
// RCCL bucket stream -- joined by events.  A missing or misplaced event would let the optimizer
// read gradients before their all-reduce finished, or update weights the scoring forward is
// still reading: a race that shows up only as slightly wrong numbers.  With
// ``NativeEngine(check_order=True)`` every stream ticks a device counter when its part of a
// step is done, and the consumers check the counters they depend on BEFORE they run:
//
//   o[0] score stream done   o[1] comm stream done   o[2] train segments done
//   o[3] steps completed (tail)   o[4] violations   o[8..11] first violation (slot, seen, want, at)
//
// Counters are touched only with agent-scope atomics (the streams run on different CUs and
// XCDs; a plain load could hit a stale line in another XCD's L2).  One lane of one workgroup
// per check: a few microseconds per step, capturable in graphs (all arguments are constants).
#include "common.h"

namespace {

MA_DEV int ld_agent(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
MA_DEV int add_agent(int* p, int v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// expect o[slot] (== or >=) o[ref] * mult + add; record a violation; then optionally tick.
__global__ __launch_bounds__(64) void order_check_kernel(int* o, int slot, int ref, int mult,
                                                         int add, int ge, int tick, int at) {
  if (threadIdx.x != 0) return;
  if (slot >= 0) {
    const int v = ld_agent(o + slot);
    const int want = ld_agent(o + ref) * mult + add;
    const bool ok = ge ? v >= want : v == want;
    if (!ok && add_agent(o + 4, 1) == 0) {
      __hip_atomic_store(o + 8, slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 9, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 10, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 11, at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tick >= 0) add_agent(o + tick, 1);
}

}  // namespace

void order_check_launch(int* o, int slot, int ref, int mult, int add, int ge, int tick, int at,
                        hipStream_t st) {
  hipLaunchKernelGGL(order_check_kernel, dim3(1), dim3(64), 0, st, o, slot, ref, mult, add, ge,
                     tick, at);
}

