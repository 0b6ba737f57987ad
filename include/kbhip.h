/*
 * kbhip.h — C ABI of libkbhip.so, the MI355X (gfx950) placement engine for
 * kube-batch's allocate action.
 *
 * The reference has no FFI: its hot path is a set of Go function types that
 * plugins register into a framework.Session.  A per-(task, node) callback
 * across cgo would cost N*T crossings, so the boundary is a batched session
 * engine called once per job pop.  Each entry point below
 * names the reference interface it replaces:
 *
 *   kbhip_session_open   <- framework.OpenSession -> cache.Snapshot()
 *                           (pkg/scheduler/framework/framework.go:29-51,
 *                            pkg/scheduler/cache/cache.go:515-583): the session
 *                           snapshot, serialised as a KBS1 buffer (kbsnap.h),
 *                           is copied, dictionary-encoded and uploaded to HBM.
 *   kbhip_place_job      <- the inner loop of allocateAction.Execute
 *                           (pkg/scheduler/actions/allocate/allocate.go:110-196)
 *                           for one job pop: per task, Session.PredicateFn
 *                           (framework/session_plugins.go:331-348, the
 *                           predicates plugin predicates.go:123-203), Session.
 *                           NodeOrderFn (:350-370, nodeorder.go:252-317),
 *                           util.SelectBestNode (util/sort.go:25-37), the
 *                           fit walk (allocate.go:149-185), Session.Allocate /
 *                           Pipeline node updates (framework/session.go:199-297)
 *                           and the gang JobReadyFn stop (gang.go:63-66).
 *   kbhip_allocate       <- allocateAction.Execute as a whole
 *                           (allocate.go:41-201) with the host-side ordering
 *                           plugins (priority, gang, drf, proportion) run by
 *                           the library's C++ mirror of the Go framework — for
 *                           callers without a Go host (bench, tests).
 *   kbhip_session_close  <- framework.CloseSession (framework.go:53-61).
 *
 * Conventions: every function returns 0 (or a count) on success and a
 * negative KBHIP_E* code on failure; nothing throws or aborts across the ABI.
 * kbhip_last_error() describes the last failure on the calling thread.
 * Inputs are caller-owned and copied; outputs are caller-allocated; the
 * session handle is engine-owned.  One session per calling thread; no host
 * thread of the library outlives a call (kbhip_session_open splits its pod
 * pass over up to 8 worker threads it joins before returning).  Device
 * memory, pinned buffers and streams of a closed session go back to a
 * process-wide pool and serve later sessions.
 *
 * Deviations from SURVEY.md §8(b)'s sketch: kbhip_session_open takes one KBS1
 * buffer that carries the plugin conf too (tiers, nodeorder arguments) instead
 * of separate kb_snapshot / kb_conf structs; node-array sharding over GPUs is
 * kbhip_session_open_shard (rank, world) instead of an n_gpus argument; the
 * open splits its pod pass over worker threads (above).
 *
 * The library has exactly one execution path: HIP on a gfx950 device.  With
 * no usable device every call fails with KBHIP_ENODEV; there is no CPU
 * fallback.
 */
#ifndef KBHIP_H_
#define KBHIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KBHIP_OK 0
#define KBHIP_EINVAL (-1)       /* malformed snapshot or arguments */
#define KBHIP_ENODEV (-2)       /* no HIP device / HIP runtime failure */
#define KBHIP_EUNSUPPORTED (-3) /* snapshot uses a feature the engine does not implement */
#define KBHIP_EDEVICE (-4)      /* kernel or copy failed */

/* placement kinds (TaskStatus after the decision) */
#define KBHIP_ALLOCATED 1 /* Session.Allocate -> api.Allocated */
#define KBHIP_PIPELINED 2 /* Session.Pipeline -> api.Pipelined */
#define KBHIP_EVICTED 3   /* Session.Evict / a committed Statement.Evict -> api.Releasing (cache.Evict) */

/* stop reasons of kbhip_place_job */
#define KBHIP_STOP_ALL 0        /* every given task was placed, job not yet ready */
#define KBHIP_STOP_UNASSIGNED 1 /* a task found no node: allocate.go:187-189 */
#define KBHIP_STOP_READY 2      /* JobReady after a placement: allocate.go:191-195 */

typedef struct kb_session kb_session;

/* Engine statistics (cumulative per session). */
typedef struct kbhip_stats {
    double open_s;       /* decode + encode + upload */
    double allocate_s;   /* wall time inside kbhip_allocate */
    double device_s;     /* summed HIP-event duration of the timed sweep launches */
    int64_t pops;        /* job pops */
    int64_t tasks;       /* tasks tried */
    int64_t placed;      /* Allocated + Pipelined */
    int64_t sweeps;      /* full-node sweeps launched */
    int64_t batched_pops;/* pops served by the class-batched path */
    int64_t nodes;       /* nodes in the session */
    int64_t timed_launches; /* sweep launches timed with HIP events (option "time_every") */
    double host_launch_s;   /* host time spent launching batched pop kernels */
    double host_wait_s;     /* host time spent waiting for their results */
    int64_t spec_hits;      /* predicted next pops launched ahead and used (kbhip_allocate) */
    int64_t spec_missed;    /* predicted pops retracted (their node updates undone on device) */
    double alloc_device_s;  /* HIP-event span of kbhip_allocate's device work (first launch to idle) */
    int64_t unassigned_pops; /* job pops that stopped on a task with no node (allocate.go:187-189) */
    int64_t collectives;     /* node-array shards: cross-shard all-gathers + all-reduces issued */
    int64_t rank_requests;   /* reclaim / preempt node rankings served by the what-if batcher ("rank_group") */
    int64_t rank_batch_sum;  /* sum over those of the sessions in the launch that served it */
    int64_t pop_requests;    /* batched allocate pops served by the what-if batcher ("rank_group") */
    int64_t pop_batch_sum;   /* sum over those of the sessions in the launch that served it */
    int64_t comm_reused;     /* 1: kbhip_shard_connect_rccl took a pooled communicator of an earlier session */
    int64_t async_launched;  /* kbhip_place_job_submit: pops launched ahead of their wait */
    int64_t async_retracted; /* ... launches withdrawn (cancelled, or behind a pop that ran synchronously) */
    int64_t async_cancelled; /* tickets withdrawn by kbhip_place_job_cancel */
    int64_t sweep_requests;  /* per-task chunks (allocate's general path, backfill) served by the what-if batcher */
    int64_t sweep_batch_sum; /* sum over those of the sessions per launch that served them */
    double score_sweep_s;    /* kbhip_sweep_scores with "time_every" > 0: summed HIP-event duration of its
                                standalone predicate + score sweep kernel (k_score_sweep) */
    int64_t score_sweeps;    /* ... launches timed */
    int64_t pertask_sweeps;  /* tasks swept one launch each (the general path: k_sweep_argmax) */
    int64_t seq_launches;    /* batched pops with a sequential placement (6: Backfilled nodes, 7: pod affinity) */
    int64_t seq_cut;         /* ... that ended before their chunk (a node outside the list could win next) */
    int64_t seq_none;        /* ... that placed nothing (the task went to the general path) */
    double evict_rank_s;     /* reclaim / preempt: host wall time in the node rankings (device sweep + copy) */
    double evict_walk_s;     /* reclaim / preempt: host wall time walking the ranked nodes (victims, evictions) */
    int64_t evict_visits;    /* reclaim / preempt: nodes whose victims were asked for (Reclaimable / Preemptable) */
    int64_t evict_cands;     /* ... candidates handed to those calls */
    int64_t fit_syncs;       /* allocate: FitDelta histograms recounted after a pop (a job left not Ready) */
    double alloc_setup_s;    /* allocate: host time before the first pop (plugin open, job and queue heaps) */
    double evict_setup_s;    /* reclaim / preempt: host time before the first node ranking (plugin open, node
                                task lists, victim codes, job heaps); part of evict_walk_s */
    int64_t engine_pops;     /* batched pops served by the persistent pop engine (option "engine") */
    int64_t engine_launches; /* launches of the engine's resident grid (one per run of engine pops) */
    int64_t engine_workers;  /* its worker blocks (0: the engine was not used) */
    int64_t engine_owners;   /* list mode (option "engine_lists"): its class-owner blocks (0: sweep mode) */
    int64_t engine_not_resident; /* engine grids that could not become resident (other kernels held CUs)
                                    and were started again */
} kbhip_stats;

/* Library / device probe: returns the number of usable gfx950 devices (>= 0),
 * or KBHIP_ENODEV when the HIP runtime is unusable. */
int kbhip_device_count(void);

/* Open a session from a KBS1 snapshot held in memory (or a file). */
int kbhip_session_open(const void* kbs_bytes, size_t len, int device, kb_session** out);
int kbhip_session_open_file(const char* path, int device, kb_session** out);

/* Place one job pop: tasks (pod indices of the snapshot, already in
 * TaskOrderFn order) are tried in sequence until one is unassigned, the job
 * becomes ready, or the list is exhausted.
 *   gang_mode      1 = the gang JobReadyFn decides, 0 = no JobReadyFn (always Ready)
 *   min_available  JobInfo.MinAvailable
 *   ready_count    tasks of the job currently in AllocatedStatuses
 * Outputs per consumed task: out_node (node index, -1 unassigned), out_kind
 * (KBHIP_ALLOCATED / KBHIP_PIPELINED / 0).  *out_n_done = tasks consumed
 * (including an unassigned one), *out_stop_reason = KBHIP_STOP_*. */
int kbhip_place_job(kb_session* s, const int32_t* task_ids, int32_t n_tasks, int32_t gang_mode,
                    int32_t min_available, int32_t ready_count, int32_t* out_node, uint8_t* out_kind,
                    int32_t* out_n_done, int32_t* out_stop_reason);

/* Asynchronous per-pop entry points: the pipelining kbhip_allocate does
 * internally, for a host that keeps allocate.go's loop
 * (allocate.go:110-196) itself.  While pop e runs, the host predicts pop e+1
 * (assuming e places its tasks as Allocated up to the gang stop), submits it,
 * and only then waits for e; if e's results show the prediction wrong, it
 * cancels e+1 and submits the real next pop.
 *
 * kbhip_place_job_submit queues one job pop with kbhip_place_job's arguments
 * and returns a ticket (>= 0).  A pop runs on the session state that every
 * earlier submitted pop leaves, exactly as a sequence of kbhip_place_job calls
 * would: a pop that is one batched chunk (at most 64 tasks, kMaxChunk, of one
 * task class) is launched at once, up to 4 ahead of the oldest wait; any other pop, and
 * every pop behind it, is launched when the pops ahead of it have been waited
 * for, or runs inside its own wait.
 * kbhip_place_job_wait returns the results of the OLDEST outstanding ticket
 * (outputs as kbhip_place_job); naming any other ticket is KBHIP_EINVAL.
 * kbhip_place_job_cancel withdraws `ticket` and every later one: their device
 * updates are undone and they are never reported.  Returns the number
 * withdrawn.
 * Every call that runs or changes the session (actions, carry, place_job,
 * kbhip_set_option, the kbhip_shard_connect_* calls, read-backs of device
 * state) fails with KBHIP_EINVAL while tickets are outstanding; read-only host
 * queries (kbhip_get_stats, kbhip_gang_unschedulable, kbhip_debug_table) are
 * allowed; kbhip_session_close drops them.
 * KBHIP_EUNSUPPORTED on node-sharded sessions (world > 1): a shard's launch
 * waits inside the cross-rank exchange and a retraction would need every rank
 * to cancel identically; shards use kbhip_place_job. */
int64_t kbhip_place_job_submit(kb_session* s, const int32_t* task_ids, int32_t n_tasks, int32_t gang_mode,
                               int32_t min_available, int32_t ready_count);
int kbhip_place_job_wait(kb_session* s, int64_t ticket, int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done,
                         int32_t* out_stop_reason);
int kbhip_place_job_cancel(kb_session* s, int64_t ticket);

/* Run the whole allocate action.  Outputs the placement log in decision
 * order: pod index, node index, kind.  Returns the number of placements. */
int kbhip_allocate(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap);

/* Run the backfill action (actions/backfill/backfill.go:40-70) on the
 * session's current state (normally after kbhip_allocate): every Pending task
 * with an empty InitResreq goes to the first node (lowest index) passing the
 * predicates.  Outputs the placements (all KBHIP_ALLOCATED) like
 * kbhip_allocate; returns their number. */
int kbhip_backfill(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap);

/* SURVEY §8(b) per-task entry points, for a Go host that keeps the
 * reference's own backfill / preempt loops and offloads only their sweeps.
 *
 * kbhip_first_fit <- the node loop of backfillAction.Execute
 *   (pkg/scheduler/actions/backfill/backfill.go:51-65): each task, in the
 *   given order, goes to the lowest-index node passing Session.PredicateFn and
 *   is committed with Session.Allocate (framework/session.go:237-297, including
 *   the drf / proportion AllocateFunc and the dispatch of a Ready job).
 *   out_node[i] = node index or -1.  Tasks must be Pending tasks of the
 *   session.  Returns the number placed.
 * kbhip_sweep_scores <- the PredicateFn + NodeOrderFn sweep of preempt()
 *   (pkg/scheduler/actions/preempt/preempt.go:270-287): out_keys[n]
 *   (optional, n_nodes entries) = pack_key(score, n) — score in bits 63..32
 *   biased by 2^31, (0x7fffffff - n) << 1 below — for a node that passes
 *   PredicateFn and has a NodeOrderFn score, 0 otherwise; sorting the keys
 *   descending is util.SelectBestNode's order (util/sort.go:25-37).  The
 *   session state is not changed.  Returns the number of passing nodes. */
int kbhip_first_fit(kb_session* s, const int32_t* task_ids, int32_t n, int32_t* out_node);
int kbhip_sweep_scores(kb_session* s, int32_t task_id, uint64_t* out_keys);

/* Measurement hook (bench.py's sweep roofline): kbhip_sweep_scores' sweep
 * kernel for each given task, launched back to back on the session stream
 * with no copies in between; *out_mean_us = device time per launch (one
 * HIP-event pair around the sequence, launch boundaries included).  Changes
 * nothing.  KBHIP_EUNSUPPORTED for classes with inter-pod priority terms
 * (their sweep needs a min / max prepass per task). */
int kbhip_time_sweeps(kb_session* s, const int32_t* task_ids, int32_t n, double* out_mean_us);

/* Measurement entry (config C5): the preempt node ranking
 * (PredicateFn + NodeOrderFn sweep + stable counting sort) of n what-if
 * sessions on one device as ONE multi-session launch chain (blockIdx.y =
 * session, each on its own node columns), session i for its pending task
 * task_ids[i]; launched reps times (evict 0: back to back; 2: each behind a
 * 512 MB cache-evicting read), descriptors copied to device memory (mapped 0)
 * or read in place from pinned mapped host memory (1).  *out_us = device
 * microseconds per chain (HIP events).  Classes of the one-pass counting sort
 * only (score range < 256, no inter-pod terms), else KBHIP_EUNSUPPORTED. */
int kbhip_time_rank_multi(kb_session* const* sessions, int32_t n, const int32_t* task_ids, int32_t reps,
                          int32_t evict, int32_t mapped, double* out_us);

/* Run the reclaim action (actions/reclaim/reclaim.go:41-196) / the preempt
 * action (actions/preempt/preempt.go:43-353) on the session's current state.
 * Output records in decision order: (pod, node, KBHIP_EVICTED) for every
 * eviction that reaches the cache (reclaim: each ssn.Evict; preempt: the
 * evictions of a committed Statement, in operation order) and
 * (pod, node, KBHIP_PIPELINED) for every pipelined preemptor (reclaim: each
 * ssn.Pipeline; preempt: those of a committed Statement).  Discarded
 * statements leave no record (and, like the reference, leave the victims'
 * node copies Releasing).  Returns the record count.  On node-sharded
 * sessions every rank calls it collectively and returns the same records:
 * each rank ranks its own nodes, the sorted lists are all-gathered
 * (kbhip_shard_connect_host_gather or kbhip_shard_connect_rccl is required,
 * else KBHIP_EINVAL) and merged, and evictions / pipelines change the rows of
 * the owning rank only.
 * Replaces the reference's reclaimAction.Execute / preemptAction.Execute.
 * If an action fails part-way (negative return) the session's host model may
 * hold a partial action: close it and open a new one. */
int kbhip_reclaim(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap);
int kbhip_preempt(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap);

/* Carry the session over to the next scheduling session (SURVEY §8(f) row 3,
 * the delta path of cache.go:515-583's per-session Snapshot): the state the
 * scheduler cache holds once this session's binds and evictions reached it —
 * dispatched tasks Bound on their nodes, Allocated-not-dispatched and
 * Pipelined tasks Pending again, evicted pods Releasing — with node rows
 * recomputed on the host and only the changed row runs uploaded (no snapshot
 * parse, no re-encode).  The session can then run its actions again.
 * *out_uploaded_bytes (optional) = bytes sent to the device.  Pod
 * (anti-)affinity count tables are recounted from the carried pod states.
 * On a node-sharded session every rank carries (identically on its
 * replicated host model; each uploads its own rows; no collective).  Pod
 * arrivals, node and PodGroup changes: kbhip_session_carry_snapshot. */
int kbhip_session_carry(kb_session* s, int64_t* out_uploaded_bytes);

/* kbhip_session_carry plus the scheduler cache's events on existing pods
 * between the two sessions (pkg/scheduler/cache/event_handlers.go), applied
 * in order after the carry:
 *   KBHIP_EV_DELETE — deletePod -> deleteTask on NewTaskInfo(pod)
 *     (event_handlers.go:119-165).  A pod of a PodGroup leaves its job and
 *     its node.  A group-less pod's TaskInfo has an empty Job
 *     (api/job_info.go:60-70), so the cache keeps it in its shadow job with
 *     its status and NodeName and only takes it off its node (the pod is
 *     "detached", kbsnap.h p_detached: it still counts for its job's
 *     readiness and the drf / proportion shares; a pending one is allocated
 *     again).  No job is deleted (JobTerminated needs a nil PodGroup).
 *   KBHIP_EV_SUCCEEDED / KBHIP_EV_FAILED — updatePod to a terminal phase
 *     (isTerminated: the task stays in its job, its node no longer counts it).
 * pods[i] are pod indices of the opened snapshot (they stay the session's pod
 * ids; a deleted pod never appears in a later record).  Every event is
 * validated first (KBHIP_EINVAL: index out of range, unknown event, an event
 * on a deleted or detached pod; KBHIP_EUNSUPPORTED: detaching a pod in a
 * session with pod (anti)-affinity terms — the predicate lister's
 * NodeInfo.Filter would leave it out at its own node only) and nothing
 * changes on error. */
enum { KBHIP_EV_DELETE = 1, KBHIP_EV_SUCCEEDED = 2, KBHIP_EV_FAILED = 3 };

/* The next scheduling session from the scheduler cache's snapshot of it
 * (cache.go:515-583 after the informer events of event_handlers.go: pod
 * arrivals, deletions and phase changes, node add / update / delete, PodGroup
 * and queue add / update), re-deriving only what changed.  kbs: the new KBS1
 * snapshot (canonical order, kbsnap.h); old_pod[i] / old_node[n]: the index
 * in THIS session of the new snapshot's pod i / node n, -1 for a new object
 * (a pod whose spec or labels changed — updatePod re-adds it, event_handlers.go
 * :101-110 — is new too).  Afterwards the session's pod and node indices are
 * the new snapshot's.  Fast path when the node set, node labels / taints and
 * the conf are unchanged, no pod carries pod (anti-)affinity terms and new
 * pods have no host ports, nodeSelector or node affinity: mapped pods keep
 * their dictionary ids and task classes, new pods are classed against the
 * kept dictionaries, jobs / queues / plugin state and node rows are
 * re-derived, and only node rows that differ (plus grown class tables) are
 * uploaded.  Any other change re-opens the session in place (same handle,
 * same options; *out_uploaded_bytes = -1).  KBHIP_EUNSUPPORTED on
 * node-sharded sessions; KBHIP_EINVAL for a malformed map.  On error the
 * session may hold a partial state: close it. */
int kbhip_session_carry_snapshot(kb_session* s, const void* kbs, size_t len, const int32_t* old_pod,
                                 const int32_t* old_node, int64_t* out_uploaded_bytes);
int kbhip_session_carry_events(kb_session* s, const int32_t* pods, const uint8_t* events, int64_t n,
                               int64_t* out_uploaded_bytes);

/* Read the device node state: N x 12 int64 (idle, used, releasing,
 * backfilled; cpu/mem/gpu each) of the session's nodes (a shard session: its
 * range [lo, hi) only).  `used` is maintained on the host mirror. */
int kbhip_read_nodes(kb_session* s, int64_t* out, int64_t n_nodes);

int kbhip_get_stats(kb_session* s, kbhip_stats* out);

/* Engine knobs: "batched" = 0 forces the per-task sweep path (tests);
 * "time_every" = k times every k-th sweep launch with HIP events;
 * "bf_batch" = 1 (default) batches pops in sessions with Backfilled nodes
 * (placement 6), 0 = per-task sweeps there;
 * "aff_batch" = 1 (default) batches pops of pod anti-affinity classes
 * (placement 7), 0 = per-task sweeps for them;
 * "aff_fence" = 1 (default) orders a placement-7 pop behind the overlapped
 * pops before it on the device (stream events; the host keeps predicted pops
 * queued), 0 = the host drains the overlap streams first;
 * "rank_radix" = 1 orders reclaim / preempt walks with the wide-range radix
 * passes (four 8-bit counting passes over the score) instead of the one-pass
 * counting sort (tests);
 * "rank_group" = 1 makes this session one of a group of what-if sessions
 * run from concurrent host threads: their allocate pops of placements 6 / 7,
 * their per-task chunks and their reclaim / preempt node rankings are issued
 * as shared multi-session launches (blockIdx.y = session): each request is
 * issued at once together with whatever other sessions' requests are pending
 * (no session waits for another; kbhip_stats
 * rank_batch_sum / rank_requests, pop_batch_sum / pop_requests and
 * sweep_batch_sum / sweep_requests (per-task chunks: allocate's general path
 * and backfill first-fits, k_sweep_argmax_multi) = requests
 * per launch);
 * "rank_first" = k: reclaim / preempt read the first k sorted keys with the count;
 * "keys32" = 1 (default) uses 32-bit selection keys in the batched sweep
 * when the class's score range and the node count fit (same order as the
 * 64-bit key), 0 = always 64-bit;
 * "speculate" = 4 (default) lets kbhip_allocate queue up to that many
 * predicted next job pops behind the running one (0..6; each used only if it
 * is exactly the next pop, retracted on device otherwise: placements are
 * unchanged), 0 = one pop at a time;
 * "engine" = 1 (default) serves eligible batched pops with the persistent pop
 * engine (one resident kernel, a descriptor ring), 0 = launched kernels;
 * "engine_workers" = n caps its worker blocks (0: as many as stay resident);
 * "engine_groups" = g its merger blocks (-1: automatic, 0: none);
 * "engine_lists" = 1 runs the engine in list mode when every eligible class
 * fits (one owner block per task class keeps the class's key of every node,
 * updated from the rows each pop touches), 0 (default) =
 * sweep mode (worker blocks sweep every node per pop);
 * "overlap" = k rotates batched pops over k + 1 streams so that a pop's sweep
 * runs beside the previous k pops' placements, chained on the device (1, the
 * default, or 2); 0 = one stream, one pop kernel at a time;
 * "shard_overlap" = 1 (node-array shards with peer mailboxes and "overlap" >
 * 0): a shard's sweep of pop e runs beside pop e-1's placement, leaving that
 * pop's candidates out and re-evaluating them once its write-back is done;
 * 0 (default) = sweep, exchange and placement one after another;
 * "debug_keys" = 1 records every per-task sweep's per-node keys (tests,
 * read back with kbhip_debug_table "dbg_keys" / "dbg_pods").
 * Measurement and rehearsal options (not part of a scheduler's use):
 * "sweep_variant" = 0..6 the kernel shape of kbhip_sweep_scores (process-wide;
 * 0 default, 4..6 grid-stride forms);
 * "time_sweeps_cold" = 0 warm, 1 write-evict, 2 read-evict the caches before
 * each launch kbhip_time_sweeps times;
 * "group_linger_us" = t (process-wide, tests) keeps a what-if batch open for
 * up to t µs for more sessions' requests;
 * "cu_split" = part * 256 + parts runs this session's streams on CUs
 * [part * C / parts, (part + 1) * C / parts) of the device's C (one-GPU
 * rehearsals of node-array shards).  "time_sweeps_cold" and
 * "cu_split" are not kept across the re-open of
 * kbhip_session_carry_snapshot's slow path. */
int kbhip_set_option(kb_session* s, const char* key, int64_t value);

/* The gang plugin's OnSessionClose after kbhip_allocate (plugins/gang/gang.go:
 * 166-187): the PodGroup Unschedulable condition message of every job that
 * is not Ready — "<m>/<n> tasks in gang unschedulable: <JobInfo.FitError>"
 * (job_info.go:343-372), the FitError from the job's NodesFitDelta as
 * allocate.go:124-126 / 164-167 leave it — one line "<job uid>\t<message>\n"
 * per job, in job UID order; empty when the gang plugin is not in the tiers.
 * Returns the text length; copies it (NUL-terminated) when cap > length. */
int64_t kbhip_gang_unschedulable(kb_session* s, char* out, int64_t cap);

int kbhip_session_close(kb_session* s);

/* Node-array sharding (one process per GPU).  A shard session
 * holds the whole host model but only nodes [lo, hi) of the snapshot on its
 * device, lo = N*rank/world, hi = N*(rank+1)/world (world <= 16).  Every rank
 * runs the same host loop; placements equal the one-GPU session's.
 *   Batched pops (the common case): each shard sweeps its range to its top-64
 *   candidates with their rows; ONE all-gather per pop exchanges them; every
 *   shard runs the identical chunk placement on the merged list (the global
 *   top-64) and writes back the rows it owns.
 *   Per-task pops (pod-affinity classes, Backfilled nodes): the 8-byte
 *   selection key (and the inter-pod affinity min/max) is all-reduced per task.
 * Connect with RCCL (kbhip_rccl_unique_id on one rank, shared out of band, then
 * kbhip_shard_connect_rccl on every rank, collectively: all-gather and
 * all-reduce on the session stream) or with host callbacks (e.g.
 * torch.distributed over gloo): kbhip_shard_connect_host for the all-reduce
 * and kbhip_shard_connect_host_gather for the all-gather; without the latter
 * every pop takes the per-task path. */
#define KBHIP_RED_MAX_U64 0
#define KBHIP_RED_MIN_I64 1
#define KBHIP_RED_MAX_I64 2
#define KBHIP_RED_SUM_I64 3 /* FitDelta counts of a task's walk over the shards */
typedef int (*kbhip_allreduce_fn)(void* ctx, uint64_t* vals, int32_t n, int32_t op);
/* recv <- the `bytes` sent by every rank, concatenated in rank order */
typedef int (*kbhip_allgather_fn)(void* ctx, const void* send, void* recv, int64_t bytes);
int kbhip_session_open_shard(const void* kbs_bytes, size_t len, int device, int32_t rank, int32_t world,
                             kb_session** out);
int kbhip_shard_info(kb_session* s, int32_t* out_rank_world_lo_hi);
int kbhip_rccl_unique_id(void* out, int64_t cap);
/* kbhip_shard_connect_rccl forms the session's communicator with a new
 * ncclCommInitRank, or takes the one a closed earlier session of this process
 * left with the same unique id, rank, world and device (communicators are
 * pooled for the process's lifetime: reuse one unique id across scheduling
 * cycles and the bootstrap is paid once; every rank must then reuse together;
 * kbhip_stats.comm_reused says which happened).  A session on which an ABI
 * call failed while it was connected, or whose communicator reports an
 * asynchronous error, aborts the communicator at close instead of pooling it. */
int kbhip_shard_connect_rccl(kb_session* s, const void* unique_id, int64_t len);
int kbhip_shard_connect_host(kb_session* s, kbhip_allreduce_fn fn, void* ctx);
/* Peer mailboxes for the batched pops of a shard session (SURVEY §8(e)'s
 * device-side exchange): every rank's device holds a mailbox (exportable
 * device memory, uncached where the runtime allows); fn all-gathers the
 * ranks' IPC handles once (every rank calls this collectively), each rank
 * maps the others' (hipIpcOpenMemHandle: xGMI across GPUs, the same memory for
 * ranks sharing one GPU).  Per batched pop every shard's sweep kernel writes
 * its top-64 with rows into every rank's mailbox and raises a flag; each
 * rank's placement kernel waits for the W flags on the device — no host
 * step and no collective launch per pop.  Takes precedence over the RCCL /
 * host all-gather for batched pops; per-task pops still use the all-reduce
 * of kbhip_shard_connect_rccl / kbhip_shard_connect_host.  Mailboxes and
 * mappings are kept per process and reused by later sessions. */
int kbhip_shard_connect_mailbox(kb_session* s, kbhip_allgather_fn fn, void* ctx);
/* Ranks that are threads of one process on one device (a rehearsal; one
 * process per GPU is the deployment): a rank's placement kernel spins on the
 * other ranks' flags, so their chained kernels must never share a hardware
 * queue.  kbhip_shard_connect_mailbox returns KBHIP_EUNSUPPORTED (every rank
 * of the group, after the all-gather) unless all ranks' streams fit in the
 * process's queues (GPU_MAX_HW_QUEUES, default 4).  This query gives the
 * same verdict without a device: 1 when ranks_on_device ranks fit in
 * hw_queues queues (hw_queues <= 0: the environment's), else 0. */
int kbhip_shard_mailbox_fits(int32_t ranks_on_device, int32_t hw_queues);
int kbhip_shard_connect_host_gather(kb_session* s, kbhip_allgather_fn fn, void* ctx);

/* Test support (not part of the placement path): encode a snapshot without a
 * device and read the compiled host tables back by name.  Tables (int32):
 *   "dims"       n_nodes, npad, n_spaces, n_classes
 *   "pod_class"  task class of every pod (-1: not a pending task)
 *   "class_aff"  per class 16 fields: aff, pred_err, ea_off, ea_n, pa_space,
 *                pa_cnt, pa_total, pa_self, paa_space, paa_cnt, ipa_off, ipa_n,
 *                upd_off, upd_n, score_err, 0
 *   "aff_dom"    [n_spaces][npad] topology domain ids
 *   "aff_cnt", "aff_scalar", "aff_items"  pod-affinity count tables / programs
 * kbhip_debug_table returns the table size in bytes and copies it when
 * cap_bytes is large enough.  Sessions from kbhip_debug_encode reject every
 * call that needs a device (KBHIP_EINVAL). */
int kbhip_debug_encode(const void* kbs_bytes, size_t len, kb_session** out);
int64_t kbhip_debug_table(kb_session* s, const char* name, void* out, int64_t cap_bytes);
/* Test support: replay a given decision sequence on an encode-only session's
 * host tables with the kernels' own per-node arithmetic (kbhip_eval.h).  Step
 * i tries task pods[i] (modes[i]: 0 allocate, 1 backfill): the selection key
 * of every node, as the device sweep computes it before the step's commit, is
 * written to out_keys[i * n_nodes + node]; then nodes[i] (-1: unassigned) is
 * committed with kinds[i] (KBHIP_ALLOCATED / KBHIP_PIPELINED).  No placement
 * decision is made here: the sequence comes from the caller (the tests take
 * it from the CPU oracle and compare the keys with the oracle's). */
int kbhip_debug_replay(kb_session* s, int32_t n_steps, const int32_t* pods, const int32_t* modes,
                       const int32_t* nodes, const uint8_t* kinds, uint64_t* out_keys);

const char* kbhip_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* KBHIP_H_ */
