// qmx_streams.h — every HIP stream the native runtime creates, and which hardware queue it
// can end up on.
//
// HIP maps streams onto hardware queues from a pool per priority level: up to
// GPU_MAX_HW_QUEUES queues per level, then the least-used queue of that level is reused.
// A persistent grid holds its queue for as long as it runs, so any stream that lands on the
// same queue waits behind it: a kernel, a copy, an RCCL round, a synchronous hipMemcpy on
// the null stream.  Measured on MI355X (tools/probes/queue_probe.hip, GPU_MAX_HW_QUEUES=4,
// profiles/r6/queues/): with the grid on a normal-priority stream and 12 more streams, 2 of
// the 12 blocked behind it; with the grid on a stream of the highest priority, none did —
// in either creation order — and neither did the null stream or a copy on a stream of its own.
//
// So the runtime has two kinds of stream:
//  * Exclusive — a persistent grid's.  Created at the greatest priority, a level whose pool
//    holds nothing else of this process (RCCL and the HIP runtime create normal-priority
//    streams), so no other work can queue behind the grid.
//  * Shared — everything else (one-shot tick launches, the exchange's RCCL rounds and copies).
//
// QMX_GRID_QUEUE=shared puts grids on normal-priority streams (the round-5 behaviour: A/B and
// the probe's negative control).  stream_stats() feeds /metrics and the bench config line.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <unordered_map>

namespace qmx {

enum class StreamKind { Shared, Exclusive };

// throws std::runtime_error when HIP cannot create the stream
hipStream_t stream_create(StreamKind kind);
void stream_destroy(hipStream_t s, StreamKind kind);
// true when Exclusive streams really get a priority level of their own (QMX_GRID_QUEUE unset
// or "exclusive", and the device has more than one priority level)
bool exclusive_queues();
// live streams per kind, the per-level queue limit this process runs with, and whether every
// exclusive stream can have a queue of its own (exclusive_live <= hw_queues)
std::unordered_map<std::string, double> stream_stats();
// Test / diagnosis (tests/test_gpu_loop_grid.py): n new Shared streams each get a trivial
// kernel, and the null stream an asynchronous copy; after wait_ms, how many had completed
// (blocked = queued behind something that holds their queue, e.g. a running persistent grid).
// Never blocks on them: they are drained (up to 5 s) before their streams are destroyed.
std::unordered_map<std::string, double> stream_probe(int n, double wait_ms);

}  // namespace qmx
