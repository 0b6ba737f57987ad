// sweep_micro.hip — diagnostic microbenchmark of the batched pop kernel's
// phases on C4-shaped synthetic node columns (100k nodes, no labels / taints /
// ports, one task class).  Includes the engine's kernel translation unit, so
// the variants below run the engine's own device code.  Never used for claims:
// it only tells which phase of k_pop_batch costs what.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 sweep_micro.hip -o sweep_micro
#include "../../kube-batch-1_amd/csrc/kbhip_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace kbhip;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

// V0: empty grid (launch + dispatch cost)
__global__ __launch_bounds__(512) void v_empty(uint32_t* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0xffffff) out[0] = 1;
}
// V1: the row loads only (the sweep's bytes), a wave max of a checksum
__global__ __launch_bounds__(512) void v_loads(NodeCols nc, uint64_t* out) {
    const int n = blockIdx.x * 512 + threadIdx.x;
    uint64_t v = 0;
    if (n < nc.n) {
        const Row r = load_row(nc, n);
        v = (uint64_t)(r.idle_cpu ^ r.idle_mem ^ r.idle_gpu ^ r.rel_cpu ^ r.rel_mem ^ r.rel_gpu ^ r.bf_cpu ^ r.bf_mem ^
                       r.bf_gpu ^ r.acpu ^ r.amem ^ r.nzc ^ r.nzm) + (uint64_t)r.pods + (uint64_t)r.maxtasks + nc.flags[n];
    }
    v = wave_max_u64(v);
    if ((threadIdx.x & 63) == 0 && v == 0x1234567) out[blockIdx.x] = v;
}
// V2: eval_node (loads + predicates + score + key) and a wave max
__global__ __launch_bounds__(512) void v_eval(Conf cf, NodeCols nc, DevTables t, uint64_t* out) {
    const TaskClass c = t.classes[0];
    const int n = blockIdx.x * 512 + threadIdx.x;
    uint64_t k = 0;
    if (n < nc.n) {
        int32_t s;
        bool passed;
        k = eval_node(cf, c, t, nc, n, &s, &passed);
    }
    k = wave_max_u64(k);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = k;
}
// V3: eval + 32-bit key + wave sort + block tree merge + list store (the per-block phase)
__global__ __launch_bounds__(512) void v_block(Conf cf, NodeCols nc, DevTables t, PopArgs a, uint32_t* out) {
    __shared__ uint32_t wlk[8][64];
    const TaskClass c = t.classes[0];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = blockIdx.x * 512 + threadIdx.x;
    uint32_t k = 0;
    if (n < nc.n) {
        int32_t s;
        bool passed;
        k = sweep_key<uint32_t>(eval_node(cf, c, t, nc, n, &s, &passed), a);
    }
    wlk[wave][lane] = wave_sort_desc(k);
    __syncthreads();
    block_tree_merge(wlk, wave, lane);
    if (wave == 0) out[blockIdx.x * 64 + lane] = wlk[0][lane];
}
// V4: V2 with the TaskClass passed by value (kernel argument) instead of loaded
__global__ __launch_bounds__(512) void v_eval_arg(Conf cf, NodeCols nc, DevTables t, TaskClass c, uint64_t* out) {
    const int n = blockIdx.x * 512 + threadIdx.x;
    uint64_t k = 0;
    if (n < nc.n) {
        int32_t s;
        bool passed;
        k = eval_node(cf, c, t, nc, n, &s, &passed);
    }
    k = wave_max_u64(k);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = k;
}

template <typename T>
static T* dev(const std::vector<T>& v) {
    T* p = nullptr;
    CK(hipMalloc(&p, std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (!v.empty()) CK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 100000;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
    const int npad = (N + 255) / 256 * 256;
    srand(7);
    const int64_t GI = 1LL << 30;
    std::vector<int64_t> ic(npad), im(npad), ig(npad), z(npad, 0), ac(npad), am(npad), nzc(npad), nzm(npad);
    std::vector<int32_t> pods(npad, 2), maxt(npad, 110);
    std::vector<uint8_t> flags(npad, 0);
    for (int i = 0; i < N; ++i) {
        const int sku = rand() % 10;
        ac[i] = sku < 3 ? 32000 : sku < 8 ? 64000 : 96000;
        am[i] = (sku < 3 ? 128 : sku < 8 ? 256 : 512) * GI;
        const int64_t uc = 500 * (1 + rand() % 8), um = GI * (1 + rand() % 8);
        ic[i] = ac[i] - uc; im[i] = am[i] - um; ig[i] = sku >= 8 ? 8000 : 0;
        nzc[i] = uc; nzm[i] = um;
    }
    NodeCols nc{};
    nc.idle_cpu = dev(ic); nc.idle_mem = dev(im); nc.idle_gpu = dev(ig);
    nc.rel_cpu = dev(z); nc.rel_mem = dev(z); nc.rel_gpu = dev(z);
    nc.bf_cpu = dev(z); nc.bf_mem = dev(z); nc.bf_gpu = dev(z);
    nc.acpu = dev(ac); nc.amem = dev(am); nc.nzc = dev(nzc); nc.nzm = dev(nzm);
    nc.pods = dev(pods); nc.maxtasks = dev(maxt); nc.flags = dev(flags);
    nc.labels = dev(std::vector<int32_t>(npad, -1)); nc.taints = dev(std::vector<uint64_t>(npad, 0));
    nc.ports = dev(std::vector<uint64_t>(npad, 0)); nc.dom = dev(std::vector<int32_t>(npad, -1));
    nc.n = N; nc.npad = npad; nc.n_keys = 0; nc.taint_words = 0; nc.port_words = 0; nc.base = 0; nc.dom_stride = npad;
    TaskClass c{};
    c.ireq_cpu = c.req_cpu = 2000; c.ireq_mem = c.req_mem = 4 * GI; c.nz_cpu = 2000; c.nz_mem = 4 * GI;
    c.nsel_term = -1; c.req_term_n = -1; c.pa_space = c.paa_space = -1;
    DevTables t{};
    t.classes = dev(std::vector<TaskClass>{c});
    t.terms = dev(std::vector<Term>(1)); t.reqs = dev(std::vector<Req>(1)); t.vals = dev(std::vector<int32_t>(1));
    t.valint = dev(std::vector<int64_t>(1)); t.valok = dev(std::vector<uint8_t>(1)); t.masks = dev(std::vector<uint64_t>(4, 0));
    t.aff_items = dev(std::vector<int32_t>(1)); t.aff_cnt = dev(std::vector<int32_t>(1)); t.aff_scalar = dev(std::vector<int32_t>(1));
    Conf cf{1, 1, 1, 1, 1, 1};
    int ibits = 1;
    while ((1 << ibits) < N) ++ibits;
    PopArgs a{0, 36, 1, 36, 0, 1, 2, 0, ibits + 1, (1 << ibits) - 1, 1, 0};
    int R;
    const int nb = pop_blocks(N, &R);
    uint64_t *out64, *cand;
    uint32_t *out32, *arrive;
    CK(hipMalloc(&out64, (size_t)nb * 64 * 8));
    CK(hipMalloc(&out32, (size_t)nb * 64 * 4));
    CK(hipMalloc(&cand, (size_t)(nb + kMaxGroups) * 64 * 8));
    CK(hipMalloc(&arrive, (3 * kMaxGroups + 1) * 32 * 4));
    CK(hipMemset(arrive, 0, (3 * kMaxGroups + 1) * 32 * 4));
    PopOut* po;
    CK(hipMalloc(&po, sizeof(PopOut)));
#ifdef KBHIP_STAMPS
    uint64_t* st;  // every k_pop_batch launch writes stamps: the buffer exists before the first one
    const size_t ns = (size_t)nb * 4 + 16;
    CK(hipMalloc(&st, ns * 8));
    CK(set_stamp_buffer(st));
#endif
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto&& launch) {
        for (int i = 0; i < 50; ++i) launch(i);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) launch(i);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-28s %8.2f us/launch (back to back, %d launches, grid %d x 512)\n", name, ms * 1e3 / iters, iters, nb);
    };
    timeit("empty", [&](int) { hipLaunchKernelGGL(v_empty, dim3(nb), dim3(512), 0, 0, out32); });
    timeit("loads", [&](int) { hipLaunchKernelGGL(v_loads, dim3(nb), dim3(512), 0, 0, nc, out64); });
    timeit("eval", [&](int) { hipLaunchKernelGGL(v_eval, dim3(nb), dim3(512), 0, 0, cf, nc, t, out64); });
    timeit("eval_classarg", [&](int) { hipLaunchKernelGGL(v_eval_arg, dim3(nb), dim3(512), 0, 0, cf, nc, t, c, out64); });
    timeit("block (sort+merge+store)", [&](int) { hipLaunchKernelGGL(v_block, dim3(nb), dim3(512), 0, 0, cf, nc, t, a, out32); });
    timeit("k_pop_batch (full, m=36)", [&](int i) {
        PopArgs b = a;
        b.epoch = (uint32_t)(i + 2) & 0xffff;
        b.fit_set = i & 1;
        hipLaunchKernelGGL((k_pop_batch<1, uint32_t, 2>), dim3(nb), dim3(512), 0, 0, cf, nc, t, b, cand, arrive, po,
                           (ShardMsg*)nullptr);
    });
    timeit("k_pop_batch (par+insert, m=36)", [&](int i) {
        PopArgs b = a;
        b.placement = 5;
        b.epoch = (uint32_t)(i + 2) & 0xffff;
        b.fit_set = i & 1;
        hipLaunchKernelGGL((k_pop_batch<1, uint32_t, 5>), dim3(nb), dim3(512), 0, 0, cf, nc, t, b, cand, arrive, po,
                           (ShardMsg*)nullptr);
    });
    timeit("k_pop_batch (shard emit)", [&](int i) {
        PopArgs b = a;
        b.placement = 3;
        b.fit_set = i & 1;
        hipLaunchKernelGGL((k_pop_batch<1, uint32_t, 3>), dim3(nb), dim3(512), 0, 0, cf, nc, t, b, cand, arrive, po,
                           (ShardMsg*)out64);
    });
    CK(hipDeviceSynchronize());
#ifdef KBHIP_STAMPS
    {  // phase timeline of k_pop_batch (stamps, 100 MHz), one launch at a time
        std::vector<uint64_t> h(ns);
        double acc[8] = {0};
        const int reps = 300;
        for (int pl : {2, 5, 4, 3}) {
            for (auto& x : acc) x = 0;
            for (int i = 0; i < reps; ++i) {
                CK(hipMemset(st, 0, ns * 8));
                PopArgs b = a;
                b.placement = pl;
                b.epoch = (uint32_t)(i + 5000) & 0xffff;
                b.fit_set = i & 1;
                if (pl == 3)
                    hipLaunchKernelGGL((k_pop_batch<1, uint32_t, 3>), dim3(nb), dim3(512), 0, 0, cf, nc, t, b, cand,
                                       arrive, po, (ShardMsg*)out64);
                else if (pl == 2)
                    hipLaunchKernelGGL((k_pop_batch<1, uint32_t, 2>), dim3(nb), dim3(512), 0, 0, cf, nc, t, b, cand,
                                       arrive, po, (ShardMsg*)out64);
                else if (pl == 5)
                    hipLaunchKernelGGL((k_pop_batch<1, uint32_t, 5>), dim3(nb), dim3(512), 0, 0, cf, nc, t, b, cand,
                                       arrive, po, (ShardMsg*)out64);
                else
                    hipLaunchKernelGGL((k_pop_batch<1, uint32_t, -1>), dim3(nb), dim3(512), 0, 0, cf, nc, t, b, cand,
                                       arrive, po, (ShardMsg*)out64);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(h.data(), st, ns * 8, hipMemcpyDeviceToHost));
                uint64_t t0 = UINT64_MAX, smax = 0, sorted_max = 0, stored_max = 0;
                double sorted_avg = 0, stored_avg = 0;
                for (int q = 0; q < nb; ++q) {
                    t0 = std::min(t0, h[q * 4]);
                    smax = std::max(smax, h[q * 4]);
                    sorted_max = std::max(sorted_max, h[q * 4 + 1]);
                    stored_max = std::max(stored_max, h[q * 4 + 2]);
                    sorted_avg += (double)(h[q * 4 + 1] - h[q * 4]) / nb;
                    stored_avg += (double)(h[q * 4 + 2] - h[q * 4]) / nb;
                }
                const uint64_t* P = h.data() + nb * 4;
                acc[0] += (smax - t0);                      // dispatch spread of block starts
                acc[1] += sorted_avg;                       // per block: start -> swept + wave-sorted
                acc[2] += stored_avg;                       // per block: start -> block list stored
                acc[3] += (stored_max - t0);                // first start -> last list stored
                acc[4] += (double)P[4] - (double)stored_max;  // -> final merger starts (group merge tail)
                acc[5] += (double)P[0] - (double)P[4];      // final merge
                acc[6] += pl != 3 ? (double)P[3] - (double)P[0] : 0;  // placement (incl. write-back)
                acc[7] += pl != 3 ? (double)P[3] - (double)t0 : (double)P[0] - (double)t0;
            }
            const char* nm[8] = {"block start spread", "block: sweep+wave sort", "block: +merge+store",
                                 "first start -> all lists stored", "group merge tail", "final merge",
                                 "placement + write-back", "span"};
            std::printf("stamps (placement %d, us):", pl);
            for (int k = 0; k < 8; ++k) std::printf(" | %s %.2f", nm[k], acc[k] / reps / 100.0);
            std::printf("\n");
        }
    }
#endif
    return 0;
}
