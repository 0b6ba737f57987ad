// sweep_floor.hip — the latency floor under the standalone sweep (k_score_sweep,
// DESIGN.md §4.6): kernels with its grid (100 000 nodes, 256 threads x 391
// blocks), one node per thread, timed by rocprofv3 --kernel-trace --stats
// (profiles/r05_floor.sh), warm (back to back) and cold (a 512 MB write before
// each launch evicts L2 and the Infinity Cache):
//   f_empty  — dispatch + drain of the grid, no memory traffic;
//   f_loads  — the sweep's bytes only: the 113 B of each node's columns
//              (13 int64, 2 int32, 1 u8) read, an 8-byte key written;
//   f_stream — the same loads over 32 copies of the columns in one launch
//              (361 MB): what HBM gives when a launch is long enough.
// Synthetic columns; diagnostic only (no claims beyond the timings).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 sweep_floor.hip -o sweep_floor
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

struct Cols {
    const int64_t* c64[13];
    const int32_t* c32[2];
    const uint8_t* c8;
    int n, copies;
};

__global__ __launch_bounds__(256) void f_empty(uint64_t* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1;
}

__global__ __launch_bounds__(256) void f_loads(Cols c, uint64_t* out) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= c.n) return;
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) v ^= (uint64_t)c.c64[i][n];
    v += (uint64_t)c.c32[0][n] + (uint64_t)c.c32[1][n] + c.c8[n];
    out[n] = v;
}

__global__ __launch_bounds__(256) void f_stream(Cols c, uint64_t* out) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= c.n * c.copies) return;
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) v ^= (uint64_t)c.c64[i][n];
    v += (uint64_t)c.c32[0][n] + (uint64_t)c.c32[1][n] + c.c8[n];
    if (v == 0x123456789ull) out[0] = v;  // (reads only)
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 100000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 64;
    const int copies = 32;
    const size_t M = (size_t)N * copies;
    Cols c{};
    for (int i = 0; i < 13; ++i) {
        int64_t* p;
        CK(hipMalloc(&p, M * 8));
        CK(hipMemset(p, i + 1, M * 8));
        c.c64[i] = p;
    }
    for (int i = 0; i < 2; ++i) {
        int32_t* p;
        CK(hipMalloc(&p, M * 4));
        CK(hipMemset(p, 7, M * 4));
        c.c32[i] = p;
    }
    uint8_t* p8;
    CK(hipMalloc(&p8, M));
    CK(hipMemset(p8, 1, M));
    c.c8 = p8;
    c.n = N;
    c.copies = copies;
    uint64_t* out;
    CK(hipMalloc(&out, (size_t)N * 8));
    void* flush;
    const size_t fb = (size_t)512 << 20;
    CK(hipMalloc(&flush, fb));
    const int nb = (N + 255) / 256;
    const int nbs = (int)((M + 255) / 256);
    // warm: back to back
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f_empty, dim3(nb), dim3(256), 0, 0, out);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f_loads, dim3(nb), dim3(256), 0, 0, c, out);
    CK(hipDeviceSynchronize());
    // cold: each launch behind the eviction write (the write is its own kernel in the trace)
    for (int r = 0; r < reps; ++r) {
        CK(hipMemsetAsync(flush, r & 0xff, fb, 0));
        hipLaunchKernelGGL(f_loads, dim3(nb), dim3(256), 0, 0, c, out);
    }
    CK(hipDeviceSynchronize());
    // long launch: 32 copies
    for (int r = 0; r < 8; ++r) hipLaunchKernelGGL(f_stream, dim3(nbs), dim3(256), 0, 0, c, out);
    CK(hipDeviceSynchronize());
    std::printf("{\"nodes\": %d, \"reps\": %d, \"grid\": %d, \"stream_copies\": %d, \"bytes_per_node\": 113}\n", N,
                reps, nb, copies);
    return 0;
}
