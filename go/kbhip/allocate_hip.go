package kbhip

// The "allocate-hip" action: kube-batch's allocate action
// (pkg/scheduler/actions/allocate/allocate.go:41-201) with the per-task node
// loop — PredicateFn over every node, NodeOrderFn, SelectBestNode, the fit
// walk (allocate.go:110-185) — on the MI355X through libkbhip.so.  It
// implements framework.Action (pkg/scheduler/framework/interface.go:20-31)
// and is registered beside the built-in actions (actions/factory.go:28-33):
//
//	framework.RegisterAction(kbhip.New())
//
// and selected in kube-batch-conf.yaml:
//
//	actions: "reclaim, allocate-hip, backfill, preempt"
//
// The plugins keep their Session API (session_plugins.go:23-65): the
// predicates and nodeorder plugins' PredicateFn / NodeOrderFn are what the
// device evaluates (their arithmetic restated in kbhip_eval.h), gang's
// JobReadyFn is the device stop rule, and the job / queue / task order of the
// priority, gang, drf and proportion plugins is either kept here in Go (mode
// PerPop: the reference's own PriorityQueues and the plugins' order
// functions, one kbhip_place_job per job pop) or run by the library's C++
// mirror of it (mode WholeAction: kbhip_allocate, one call).  Either way every
// placement is applied through the reference's own ssn.Allocate /
// ssn.Pipeline (session.go:199-297), so JobInfo status, the plugins' event
// handlers (drf / proportion shares) and dispatch / bind stay the reference's.
//
// NOT COMPILED HERE (no Go toolchain in this image): see kbhip.go.  The same
// loops are run against the library by tests/gohost.py (Python) and
// kube-batch-1_amd/host/kbhost.cpp (C++), whose logs equal the oracle's.

import (
	"github.com/golang/glog"

	"github.com/kubernetes-sigs/kube-batch/pkg/scheduler/actions/allocate"
	"github.com/kubernetes-sigs/kube-batch/pkg/scheduler/api"
	"github.com/kubernetes-sigs/kube-batch/pkg/scheduler/framework"
	"github.com/kubernetes-sigs/kube-batch/pkg/scheduler/util"
)

// Mode selects who keeps the job / queue order.
type Mode int

const (
	WholeAction Mode = iota // kbhip_allocate: the order in the library (C++ mirror), one call
	PerPop                  // allocate.go's loop here, one kbhip_place_job per job pop
)

type allocateHIPAction struct {
	mode   Mode
	device int
}

// New returns the action (WholeAction on device 0).
func New() *allocateHIPAction { return &allocateHIPAction{mode: WholeAction} }

// NewWith returns the action with a chosen mode and device.
func NewWith(mode Mode, device int) *allocateHIPAction {
	return &allocateHIPAction{mode: mode, device: device}
}

func (a *allocateHIPAction) Name() string { return "allocate-hip" }

func (a *allocateHIPAction) Initialize() {}

func (a *allocateHIPAction) UnInitialize() {}

// Execute runs allocate on the device; if the engine cannot take the session
// (no device, an input the encoder or the engine refuses), the reference
// action runs instead — same placements, CPU speed.
func (a *allocateHIPAction) Execute(ssn *framework.Session) {
	glog.V(3).Infof("Enter Allocate (hip) ...")
	defer glog.V(3).Infof("Leaving Allocate (hip) ...")
	snap, idx, err := EncodeSession(ssn)
	var eng *Engine
	if err == nil {
		eng, err = Open(snap, a.device)
	}
	if err != nil {
		glog.Warningf("kbhip unavailable for this session (%v): running the reference allocate", err)
		allocate.New().Execute(ssn)
		return
	}
	defer eng.Close()
	if a.mode == PerPop {
		err = executePerPop(ssn, eng, idx)
	} else {
		err = executeWhole(ssn, eng, idx)
	}
	if err != nil {
		// placements applied so far stay (each went through ssn.Allocate / ssn.Pipeline);
		// the rest of the session runs on the CPU path
		glog.Errorf("kbhip: %v: finishing with the reference allocate", err)
		allocate.New().Execute(ssn)
	}
}

// apply one placement through the reference's session (allocate.go:161-181).
func apply(ssn *framework.Session, task *api.TaskInfo, host string, kind uint8) error {
	if kind == Allocated {
		// usingBackfillTaskRes: InitResreq does not fit Idle alone (allocate.go:161)
		node := ssn.Nodes[host]
		return ssn.Allocate(task, host, !task.InitResreq.LessEqual(node.Idle))
	}
	return ssn.Pipeline(task, host)
}

// executeWhole: kbhip_allocate places every pop with its C++ mirror of the
// order (priority / gang / drf / proportion, Go container/heap exact), then
// the log is applied in decision order — the same sequence of ssn.Allocate /
// ssn.Pipeline calls the reference makes, so every event handler sees the
// same states.
func executeWhole(ssn *framework.Session, eng *Engine, idx *Index) error {
	log, err := eng.Allocate(len(idx.Pods) + 1)
	if err != nil {
		return err
	}
	for _, p := range log {
		if err := apply(ssn, idx.Pods[p.Pod], idx.NodeNames[p.Node], p.Kind); err != nil {
			glog.Errorf("kbhip: placing task %v on %v: %v", idx.Pods[p.Pod].UID, idx.NodeNames[p.Node], err)
		}
	}
	return nil
}

// executePerPop: allocate.go:41-201 with the order kept here and the node
// loop of each job pop on the device (kbhip_place_job).  The gang JobReadyFn
// runs on the device as the stop rule (gang.go:63-66: ready = allocated >=
// MinAvailable); ssn.JobReady decides the heap push as in the reference.
func executePerPop(ssn *framework.Session, eng *Engine, idx *Index) error {
	queues := util.NewPriorityQueue(ssn.QueueOrderFn)
	jobsMap := map[api.QueueID]*util.PriorityQueue{}
	for _, job := range ssn.Jobs { // (map order; the snapshot pins the reference's to UID order)
		if queue, found := ssn.Queues[job.Queue]; found {
			queues.Push(queue)
		} else {
			continue
		}
		if _, found := jobsMap[job.Queue]; !found {
			jobsMap[job.Queue] = util.NewPriorityQueue(ssn.JobOrderFn)
		}
		jobsMap[job.Queue].Push(job)
	}
	gang := gangInTiers(ssn)
	pendingTasks := map[api.JobID][]*api.TaskInfo{}
	for !queues.Empty() {
		queue := queues.Pop().(*api.QueueInfo)
		if ssn.Overused(queue) {
			continue
		}
		jobs, found := jobsMap[queue.UID]
		if !found || jobs.Empty() {
			continue
		}
		job := jobs.Pop().(*api.JobInfo)
		if _, found := pendingTasks[job.UID]; !found {
			tq := util.NewPriorityQueue(ssn.TaskOrderFn)
			for _, task := range job.TaskStatusIndex[api.Pending] {
				if task.Resreq.IsEmpty() { // BestEffort: skipped by allocate
					continue
				}
				tq.Push(task)
			}
			var order []*api.TaskInfo
			for !tq.Empty() {
				order = append(order, tq.Pop().(*api.TaskInfo))
			}
			pendingTasks[job.UID] = order
		}
		tasks := pendingTasks[job.UID]
		if len(tasks) > 0 {
			ids := make([]int32, len(tasks))
			for i, t := range tasks {
				ids[i] = idx.PodIndex[t.UID]
			}
			ready := int32(len(job.GetTasks(api.AllocatedStatuses()...))) // GetReadiness (job_info.go:374-389)
			nodes, kinds, stop, err := eng.PlaceJob(ids, gang, job.MinAvailable, ready)
			if err != nil {
				return err
			}
			for i := range nodes {
				if nodes[i] < 0 {
					break // allocate.go:187-189: the first task without a node ends the pop
				}
				if err := apply(ssn, tasks[i], idx.NodeNames[nodes[i]], kinds[i]); err != nil {
					glog.Errorf("kbhip: placing task %v: %v", tasks[i].UID, err)
				}
			}
			pendingTasks[job.UID] = tasks[len(nodes):]
			if stop == StopReady && ssn.JobReady(job) {
				jobs.Push(job) // allocate.go:191-195
			}
		}
		queues.Push(queue) // allocate.go:198-199
	}
	return nil
}

func gangInTiers(ssn *framework.Session) bool {
	for _, tier := range ssn.Tiers {
		for _, p := range tier.Plugins {
			if p.Name == "gang" && !p.JobReadyDisabled {
				return true
			}
		}
	}
	return false
}
