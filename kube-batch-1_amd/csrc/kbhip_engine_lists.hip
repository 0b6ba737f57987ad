// kbhip_engine_lists.hip — the persistent pop engine in list mode (DESIGN.md
// §4.11): one owner block per task class keeps the class's key of every node
// in LDS and writes each pop's package; the placer and the dispatcher are the
// sweep engine's (engine/engine_placer.h).  Its own translation unit, so that
// the two engine kernels compile side by side.
#include <hip/hip_runtime.h>

#include "engine/engine_dev.h"
#include "engine/engine_owner.h"
#include "engine/engine_placer.h"

namespace kbhip {

// List mode: class owners, the placer, the dispatcher.  A
// kernel of its own, so that the owners' registers do not weigh on the sweep
// engine's placer.
__global__ __launch_bounds__(kPopThreads) void k_engine_lists(Conf cf, NodeCols nc, DevTables t, EngArgs A) {
    __shared__ EngLdsList lds;
    __shared__ int arrived;
    const int b = blockIdx.x;
    if (!eng_arrive(A, &arrived)) {
        if (b == A.nown + 1) eng_not_resident(A);
        return;
    }
    if (b < A.nown) eng_owner(cf, nc, t, A, lds.o, b);
    else if (b == A.nown) eng_placer<true>(cf, nc, t, A, lds.p);
    else if (threadIdx.x < 64) eng_dispatch(A);
}

hipError_t launch_engine_lists(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A, int grid,
                               hipStream_t st) {
    hipLaunchKernelGGL(k_engine_lists, dim3(grid), dim3(kPopThreads), 0, st, cf, nc, t, A);
    return hipGetLastError();
}

hipError_t engine_lists_occupancy(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_engine_lists, kPopThreads, 0);
}

}  // namespace kbhip
