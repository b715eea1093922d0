/*
 * cpu_baseline.h — CPU BASELINE FOR bench.py ONLY (test infrastructure).
 *
 * The Rust reference cannot be built in this image, so the CPU baseline is a
 * restatement of its threaded CPU path, structured like the reference:
 *  - pack: input split into max(1, T/4) chunks (src/array/operations.rs:462-480),
 *    each packed by its own thread into op buffers of ceil(am_size_threshold /
 *    sizeof(IdxVal<I,T>)) records (src/array/unsafe/operations.rs:663-811);
 *  - apply: T threads pull op buffers and apply every record with SeqCst
 *    atomics for integer elements (NativeAtomicArray: fetch_add/sub/and/or/xor,
 *    CAS loops with yield for mul/div/rem — src/array/native_atomic.rs:29-113,
 *    impl/src/array_ops.rs:327-458) and a 1-byte lock per element for f32/f64
 *    (GenericAtomicArray, src/array/generic_atomic.rs:286-293);
 *  - fetch results land in input order (src/array/operations/handle.rs:315-317).
 * One PE (the local lamellae): every op buffer targets this process's shard.
 */
#ifndef LAMELLAR_CPU_BASELINE_H
#define LAMELLAR_CPU_BASELINE_H

#include "../include/lamellar_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double pack_s;
    double apply_s;
    double total_s;
    uint64_t n_buffers;
} cpu_times_t;

/* Runs one batched op on `shard` (shard_len elements of dtype) with `threads`
 * apply threads. vals == NULL -> single value `*val` for every index.
 * results (may be NULL) receive fetch values in input order. */
int cpu_baseline_run(uint32_t dtype, uint32_t op, void* shard, uint64_t shard_len,
                     const uint64_t* gidx, const void* vals, const void* val, uint64_t n,
                     uint32_t threads, uint64_t am_size_threshold, const void* cmp, void* results,
                     cpu_times_t* out);

/* C4: npes PEs (Block layout over array_len elements) of threads_per_pe threads each,
 * exchanging op buffers through shared memory with the shmem lamellae's command-queue
 * protocol restated (see cpu_baseline.c); ops that return nothing, integer types. shards[p]
 * = PE p's shard (num_elems_pe elements), gidx[p] / vals[p] = PE p's n_per_pe records. */
int cpu_baseline_multi_pe(uint32_t dtype, uint32_t op, uint32_t npes, uint32_t threads_per_pe, uint64_t array_len,
                          void* const* shards, const uint64_t* const* gidx, const void* const* vals, uint64_t n_per_pe,
                          uint64_t am_size_threshold, cpu_times_t* out);

#ifdef __cplusplus
}
#endif
#endif
