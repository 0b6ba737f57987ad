// kbhip_engine.hip — the persistent pop engine: one
// resident grid places a run of batched job pops (allocate.go:110-185, one
// gang chunk of one task class per pop) with no kernel launch per pop.
// Roles by block (kbhip_engine.h):
//   [0, nw)        workers: node range [b * npb, (b + 1) * npb)
//   [nw, nw + ng)  mergers: group g = workers b with b % ng == g
//   nw + ng        final merger (the package of the group lists' top 128)
//   nw + ng + 1    placer
//   nw + ng + 2    dispatcher (one wave)
// Hand-offs are self-tagged 8-byte granules {seq << 32 | value} written with
// sc1 stores and polled with sc1 loads (MI355X_MICROARCH.md, R2), or sc1 row
// stores drained before the sc1 `done` flag (valid forms, table row 1).
// Every wait is bounded (s_memrealtime) and gives up once ctl->err is set.
#include <hip/hip_runtime.h>

#include "engine/engine_dev.h"
#include "engine/engine_placer.h"
#include "engine/engine_sweep.h"

namespace kbhip {

// the list-mode kernel (kbhip_engine_lists.hip)
hipError_t launch_engine_lists(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A, int grid,
                               hipStream_t st);
hipError_t engine_lists_occupancy(int* blocks_per_cu);

__global__ __launch_bounds__(kPopThreads) void k_engine(Conf cf, NodeCols nc, DevTables t, EngArgs A) {
    __shared__ EngLds lds;
    __shared__ int arrived;
    const int b = blockIdx.x;
    if (!eng_arrive(A, &arrived)) {
        if (b == A.nw + A.ng + 2) eng_not_resident(A);
        return;
    }
    if (b < A.nw) {
        eng_worker(cf, nc, t, A, lds.w, b);
    } else if (b < A.nw + A.ng) {
        eng_merger(A, lds.m, b - A.nw);
    } else if (b == A.nw + A.ng) {
        eng_final(cf, nc, t, A, lds.m);
    } else if (b == A.nw + A.ng + 1) {
        eng_placer<false>(cf, nc, t, A, lds.p);
    } else if (threadIdx.x < 64) {
        eng_dispatch(A);
    }
}

int engine_grid(const EngArgs& A) { return A.nown > 0 ? A.nown + 2 : A.nw + A.ng + 3; }

hipError_t launch_engine(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A, hipStream_t st) {
    if (A.nown > 0) return launch_engine_lists(cf, nc, t, A, engine_grid(A), st);
    hipLaunchKernelGGL(k_engine, dim3(engine_grid(A)), dim3(kPopThreads), 0, st, cf, nc, t, A);
    return hipGetLastError();
}

hipError_t engine_occupancy(int* blocks_per_cu, bool lists) {
    if (lists) return engine_lists_occupancy(blocks_per_cu);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_engine, kPopThreads, 0);
}

}  // namespace kbhip
