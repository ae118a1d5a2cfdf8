// api_lock.hpp — one process-wide lock for the library's device-wide HIP calls.
//
// A stream capture in one host thread is invalidated by a legacy-stream (synchronous) call or an
// allocation another thread makes while it is open.  The reference drives the library from one
// host thread per GPU (src/llama.cpp:919-1024) and the CLI may run several replicas per device, so
// every graph capture (begin .. instantiate) and every synchronous / allocating call the library
// makes (decoder create / destroy, RunState and arena residency, the memcpy helpers) holds this
// lock; per-call work is ordered on each decoder's own non-blocking stream and needs no lock.
#pragma once
#include <mutex>

namespace tl {
std::recursive_mutex& api_mu();
typedef std::lock_guard<std::recursive_mutex> ApiLock;
}  // namespace tl
