// Reclaim / preempt node ranking on gfx950.
//
// Both actions walk the nodes for one preemptor task in a fixed order and stop
// at the first node whose victims cover the request:
//   preempt  (actions/preempt/preempt.go:270-288): nodes passing PredicateFn
//            with a NodeOrderFn score, in util.SelectBestNode order (score
//            descending, then the pinned node order);
//   reclaim  (actions/reclaim/reclaim.go:115-119): nodes passing PredicateFn,
//            in the pinned node order.
// The victim choice itself (tier-intersected Preemptable / Reclaimable over the
// node's tasks) is per-node host logic on the host model.  The device produces
// the order: one HBM sweep writes a key per node — pack_key(score, idx) for
// preempt (descending = SelectBestNode order), pack_key(0, idx) for reclaim —
// zero for a node that fails; a device radix sort orders the keys, and the
// host reads the passing prefix back.  Traffic per task: the per-task sweep's
// B_node bytes per node + 8 B written per node + the sort's passes over 8 B keys.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "kbhip_eval.h"
#include "kbhip_internal.h"

namespace kbhip {

__global__ __launch_bounds__(kBlock) void k_rank_nodes(Conf cf, NodeCols nc, DevTables t, const PopCtrl* ctrl,
                                                       int by_score, uint64_t* keys, uint32_t* count) {
    __shared__ uint32_t s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const int cls = __builtin_amdgcn_readfirstlane(ctrl->cls[0]);
    const TaskClass c = t.classes[cls];
    const int64_t ilo = ctrl->ipa_lo[0], ihi = ctrl->ipa_hi[0];
    const int F = ctrl->fallback;
    uint32_t cnt = 0;
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        uint64_t k;
        if (by_score) {
            int32_t s = 0;
            bool passed = false;
            (void)eval_node_aff(cf, c, t, nc, n, ilo, ihi, F, &s, &passed);
            k = passed ? pack_key(s, n + nc.base, 0) : 0;
        } else {
            k = eval_first_fit(cf, c, t, nc, n);
        }
        keys[n] = k;
        cnt += k != 0;
    }
    // wave sum, then one LDS atomic per wave and one global atomic per block
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(count, s_cnt);
}

// One node-row update of a reclaim / preempt operation, in one lane:
//   op 0 evict       NodeInfo.UpdateTask Running -> Releasing: Releasing += Resreq
//                    (node_info.go:147-185; Idle / Used / Backfilled net unchanged)
//   op 1 pipeline    NodeInfo.AddTask Pipelined (commit_node, kind 2)
//   op 2 unpipeline  NodeInfo.RemoveTask of the Pipelined copy (uncommit_node, kind 2)
__global__ __launch_bounds__(64) void k_node_op(NodeCols nc, DevTables t, int op, int n, int cls, int64_t rc,
                                                int64_t rm, int64_t rg) {
    if (threadIdx.x != 0) return;
    if (op == 0) {
        nc.rel_cpu[n] += rc; nc.rel_mem[n] += rm; nc.rel_gpu[n] += rg;
    } else if (op == 1) {
        commit_node(t.classes[cls], t, nc, n, 2);
    } else {
        uncommit_node(t.classes[cls], t, nc, n, 2);
    }
}

// Accumulated evictions (op 0 of k_node_op, summed per node on the host):
// Releasing += d[3 i .. 3 i + 2] on node[i]; the nodes are distinct.
__global__ __launch_bounds__(kBlock) void k_rel_add(NodeCols nc, const int32_t* node, const int64_t* d, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int v = node[i];
    nc.rel_cpu[v] += d[3 * i]; nc.rel_mem[v] += d[3 * i + 1]; nc.rel_gpu[v] += d[3 * i + 2];
}

hipError_t launch_rel_add(const NodeCols& nc, const int32_t* node, const int64_t* d, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rel_add, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, nc, node, d, n);
    return hipGetLastError();
}

hipError_t launch_rank_nodes(const Conf& cf, const NodeCols& nc, const DevTables& t, const PopCtrl* ctrl,
                             int by_score, uint64_t* keys, uint32_t* count, hipStream_t st) {
    int grid = (nc.n + kBlock - 1) / kBlock;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_rank_nodes, dim3(grid), dim3(kBlock), 0, st, cf, nc, t, ctrl, by_score, keys, count);
    return hipGetLastError();
}

hipError_t sort_keys_desc(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out, int n, hipStream_t st) {
    return hipcub::DeviceRadixSort::SortKeysDescending(tmp, *tmp_bytes, in, out, n, 0, 64, st);
}

hipError_t launch_node_op(const NodeCols& nc, const DevTables& t, int op, int n, int cls, int64_t rc, int64_t rm,
                          int64_t rg, hipStream_t st) {
    hipLaunchKernelGGL(k_node_op, dim3(1), dim3(64), 0, st, nc, t, op, n, cls, rc, rm, rg);
    return hipGetLastError();
}

}  // namespace kbhip
