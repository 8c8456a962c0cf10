// Durability of the HBM tables: compaction of the transfer store and checkpoint images.
//
// The reference persists its state through the Forest: `compact` (state_machine.zig:2912-2935)
// runs the LSM compactions of one beat, `checkpoint` (:2937-2958) makes the compacted trees
// durable, `open` (:964-978) loads them back. Here the tables live in HBM:
//
//   * tbg_compact squeezes the transfer store. Rows are consumed by every create_transfers event
//     (an event's row is written as it ingests, executor.hip), so rows of events that created no
//     object and whose id is not orphaned are garbage. Compaction keeps exactly the rows an id
//     slot refers to (created transfers and orphaned ids), in order (row order is timestamp order,
//     which the pulse's sort and the dumps rely on), rebuilds the id index from them -- dropping
//     the tombstones of failed claims -- and renumbers every persistent row reference (the
//     expires_at index, AccountEvent references).
//   * tbg_checkpoint / tbg_open_checkpoint write and read a self-describing image of every
//     persistent table (executor.hip).
#pragma once

#include "events.hpp"

namespace tbg {

// keep32[r] = 1 for every row a slot refers to (created or orphaned), over the whole slot table.
__global__ void cmp_mark(const IdTable tr, uint64_t used, uint32_t* keep32) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i > tr.mask) return;
    const uint64_t w = tr.slots[i];
    if (w == kEmpty || w == kTomb) return;
    const uint64_t r = (w & kRefMask) - 1;
    if (r < used) keep32[r] = 1;
}

// Rows [a, b) that are kept, to their new positions relative to new_row[a] (base) in the chunk
// buffers.
__global__ void cmp_gather(const tb_transfer_t* rows, const uint8_t* live, const uint8_t* status,
                           const uint32_t* keep32, const uint32_t* new_row, uint64_t a, uint64_t b,
                           uint32_t base, tb_transfer_t* c_rows, uint8_t* c_live,
                           uint8_t* c_status) {
    const uint64_t r = a + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= b || !keep32[r]) return;
    const uint32_t j = new_row[r] - base;
    copy_row(&c_rows[j], &rows[r]);
    c_live[j] = live[r];
    c_status[j] = status[r];
}

// The id index from the kept rows: created rows as objects, the others as orphaned ids (a row a
// slot referred to and that is not live holds an orphaned id). Ids are unique: plain claims.
__global__ void cmp_insert(const IdTable tr, const tb_transfer_t* rows, const uint8_t* live,
                           uint64_t kept, unsigned int* failed) {
    const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= kept) return;
    const tb_uint128_t id = rows[r].id;
    const uint64_t w = id_tag(id) | (live[r] ? 0 : kOrphanBit) | (r + 1);
    uint64_t s = hash_id(id) & tr.mask;
    for (uint64_t n = 0; n < probe_limit(tr.mask); n++) {
        if (atomicCAS(&tr.slots[s], (unsigned long long)kEmpty, (unsigned long long)w) == kEmpty)
            return;
        s = probe_next(s, tr.mask);
    }
    atomicAdd(failed, 1u);
}

// expires_at entries whose row is kept (flags for an order-preserving selection).
__global__ void cmp_expiry_flags(const uint64_t* expiry, uint64_t count, uint64_t used,
                                 const uint32_t* keep32, uint8_t* flags) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint64_t row = expiry[i];
    flags[i] = row < used && keep32[row];
}

__global__ void cmp_expiry_gather(const uint64_t* expiry, const uint32_t* sel, uint64_t n,
                                  const uint32_t* new_row, uint64_t* out) {
    const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (j < n) out[j] = new_row[expiry[sel[j]]];
}

// AccountEvent references name created (kept) transfer rows.
__global__ void cmp_ae_refs(AeRef* refs, uint64_t n, const uint32_t* new_row) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) refs[i].transfer_row = new_row[refs[i].transfer_row];
}

}  // namespace tbg
