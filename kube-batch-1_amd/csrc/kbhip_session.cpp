// kbhip_session.cpp — host side of libkbhip.so: session open (KBS1 decode,
// dictionary encoding, upload of the node SoA to HBM), the per-pop device
// driver (kbhip_place_job) and a C++ mirror of the Go framework's ordering
// plugins that runs the whole allocate action (kbhip_allocate).
//
// Reference map (pkg/scheduler unless noted):
//   session open      cache/cache.go:515-583 (Snapshot), framework/session.go:66-122,
//                     api/node_info.go:62-145 (NodeInfo.AddTask), api/job_info.go:239-326
//   ordering          util/priority_queue.go + Go container/heap, framework/session_plugins.go:
//                     244-329 (Job/Queue/TaskOrderFn), plugins/{priority,gang,drf,proportion}
//   allocate loop     actions/allocate/allocate.go:41-201
//   placement         the HIP kernels (kbhip_kernels.hip)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <random>
#include <tuple>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <unistd.h>

#include "../../include/kbhip.h"
#include "../../include/kbsnap.h"
#include "kbhip_affinity.h"
#include "kbhip_engine.h"
#include "kbhip_eval.h"
#include "kbhip_internal.h"

using std::string;
using std::vector;


// The session's text is split by subject into csrc/session/*.inc (one
// translation unit):
#include "session/01_types.inc"
#include "session/02_open.inc"
#include "session/03_pop.inc"
#include "session/04_allocate.inc"
#include "session/05_actions.inc"
#include "session/06_carry.inc"
#include "session/07_abi.inc"
