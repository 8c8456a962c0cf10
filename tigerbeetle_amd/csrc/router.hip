// The device-side ledger router (include/tbr.h): directories and the device path of a routed call.
//
// Directories are the executor's id tables (device_common.hpp: tagged slots, group-16 homes) over
// append-only stores: accounts (id, shard) in insertion order; transfers (id, shard) per routed
// event position -- every event of a routed call takes a store row, like the executor's transfer
// rows, and its slot claim is released at settle unless the id now exists on its shard.
//
// Device path, per call of n events (one workgroup per 256 consecutive events, so the scatter is
// stable): tbr_pass1 -- the id claim and the shard the event's own fields pin (its id's holder,
// its accounts', or any shard for an event whose status follows from itself alone; surrogates for
// accounts on two shards); tbr_pass_pv -- a post/void's shard from its pending transfer;
// tbr_pass_dup -- an id repeated in the call on its first occurrence's shard; tbr_pass_chains --
// linked chains whole on one shard, events that may run anywhere placed; tbr_pass_count --
// per-block counts per shard; the host turns them into per-block offsets (shard-major exclusive
// sums); tbr_pass2 -- each event copied to its slice with its global commit timestamp and its
// position; after the shards ran: tbr_settle / tbr_settle_release -- results to call order,
// surrogate statuses patched, directory slots kept or released.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/tbr.h"
#include "replay.hpp"

using namespace tbg;

namespace {

constexpr uint32_t kRouteBlock = 256;
constexpr uint32_t kShardsMax = 64;

struct Dir {
    IdTable slots;
    tb_uint128_t* ids;
    uint8_t* shard;
};

struct RouteArgs {
    Dir acc, tr;
    const tb_transfer_t* events;
    uint32_t n;
    const uint32_t* batch_ends;
    const uint64_t* batch_ts;
    uint32_t n_batches;
    uint64_t base;          // the call's first transfer-store row
    uint32_t shards;
    uint32_t nblocks;
    uint8_t* ev_shard;      // per event: its shard, 0xFF for a hazard
    uint32_t* ev_slot;      // per event: its claimed slot (kNone32: none)
    uint8_t* ev_patch;      // per event: a surrogate's status (0: none)
    uint8_t* ev_keep;       // per first occurrence: its id exists after the call
    uint8_t* ev_link;       // per event: its linked flag (tbr_pass_chains reads no event again)
    uint32_t* ev_owner;     // per repeat: its first occurrence's position (else kNone32)
    uint32_t* block_counts; // [shard][block]
    unsigned int* flags;    // [0] hazard, [1] table full, [2] the call posts or voids,
                            // [3] bit 0: an imported event, bit 1: a non-imported one,
                            // [4] events that may run anywhere, [5] surrogates, [6] repeats
    uint64_t imported_floor;  // imported timestamps at or below it are hazards (tbr.h)
};

// A shard's slice: where the scatter writes its events and timestamps, where its executor writes
// the results, and its first position in the call's shard-major order.
struct SliceDst {
    tb_transfer_t* events;
    uint64_t* timestamps;
    const tb_create_result_t* results;
    uint64_t base;
};

__device__ inline uint64_t dir_find(const Dir& d, const tb_uint128_t& id) {
    const tb_uint128_t* ids = d.ids;
    const uint64_t s = probe_find(d.slots, id, [=](uint64_t r) { return ids[r]; });
    if (s == kNone) return kNone;
    return (d.slots.slots[s] & kRefMask) - 1;
}

__global__ void tbr_insert(Dir d, uint64_t base, uint32_t n, unsigned int* flags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tb_uint128_t* ids = d.ids;
    bool dup = false;
    const uint64_t s = probe_claim(d.slots, ids[base + i], base + i + 1, base,
                                   [=](uint64_t r) { return ids[r]; }, &dup);
    if (s == kNone) atomicOr(&flags[1], 1u);
}

__global__ void tbr_lookup(Dir d, const tb_uint128_t* q, uint32_t n, int32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t r = dir_find(d, q[i]);
    out[i] = r == kNone ? -1 : int32_t(d.shard[r]);
}

// ev_shard codes besides a shard: the event is a hazard (the call goes to the exact engine), a
// post/void whose shard follows its pending transfer (resolved by tbr_pass_pv), or an event whose
// status follows from itself alone and runs on any shard (resolved by tbr_pass_chains).
constexpr uint8_t kShardHazard = 0xFF;
constexpr uint8_t kShardPending = 0xFE;
constexpr uint8_t kShardAny = 0xFD;

// Sets bits of a call-wide flag word from one lane of the wave: tested first, so that only the
// waves that find a bit clear issue the atomic (one atomic a wave to one word serialises every
// wave of the grid in one L2 channel: ~11 ns each, 720 us over a 4M-event call).
__device__ inline void set_flag(unsigned int* word, unsigned int bits) {
    if ((__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bits) != bits)
        atomicOr(word, bits);
}
__device__ inline void raise_hazard(const RouteArgs& a, bool hazard) {
    if (__any(hazard) && (threadIdx.x & 63) == 0) set_flag(&a.flags[0], 1u);
}
__device__ inline void count_wave(unsigned int* counter, bool x) {
    const uint64_t m = __ballot(x);
    if (m && (threadIdx.x & 63) == 0) atomicAdd(counter, unsigned(__popcll(m)));
}

// create_transfer's status for a transfer whose two accounts exist on two shards (so on two
// ledgers): the first failing check after accounts_must_be_different (:3756-3798) -- none of them
// reads state, the last is accounts_must_have_the_same_ledger. (engine.hpp cross_status.)
__device__ inline uint8_t cross_status(const tb_transfer_t& t) {
    if (!u128_is_zero(t.pending_id)) return TB_CT_PENDING_ID_MUST_BE_ZERO;
    if (!(t.flags & TB_TRANSFER_PENDING)) {
        if (t.timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
        if (t.flags & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT))
            return TB_CT_CLOSING_TRANSFER_MUST_BE_PENDING;
    }
    if (t.ledger == 0) return TB_CT_LEDGER_MUST_NOT_BE_ZERO;
    if (t.code == 0) return TB_CT_CODE_MUST_NOT_BE_ZERO;
    return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
}

// The wave's 64 consecutive events staged in LDS with fully coalesced 16-byte loads (each lane
// then reads its own event's fields from LDS): 8 load instructions a wave instead of one per
// field, each touching 64 lines. 144 bytes per event: an 8-lane group writes one event's 128
// contiguous bytes, no two lanes on a bank (kernels.hpp tr_ingest).
constexpr uint32_t kStageStride = 144;
__device__ inline const tb_transfer_t* stage_wave_events(const tb_transfer_t* events, uint32_t n,
                                                         uint8_t* my) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t k0 = blockIdx.x * kRouteBlock + (threadIdx.x & ~63u);
    const uint32_t cnt = n > k0 ? (n - k0 < 64 ? n - k0 : 64) : 0;
    const uint4* src = reinterpret_cast<const uint4*>(events + k0);
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t idx = i * 64 + lane;
        v4u v = {0, 0, 0, 0};
        if (idx < cnt * 8) v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(&src[idx]));
        const uint32_t e = i * 8 + (lane >> 3), part = lane & 7;
        *reinterpret_cast<v4u*>(__builtin_assume_aligned(my + e * kStageStride + part * 16, 16)) = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return reinterpret_cast<const tb_transfer_t*>(my + lane * kStageStride);
}

// Pass 1, per event: the shard its own fields pin.
//  * A status that follows from the event alone (a nonzero padding, an id 0 / maxInt, a nonzero
//    timestamp on a non-imported event: execute_create :3080, create_transfer :3729-3732) reads
//    no state: any shard, no id claim.
//  * Otherwise the id is claimed: an id that already exists goes to its holder
//    (create_transfer_exists / id_already_failed run before any account lookup, :3733-3738); a
//    post/void waits for its pending transfer (tbr_pass_pv); a transfer goes to its accounts'
//    shard -- the known one's when the other is unknown (debit_account_not_found /
//    credit_account_not_found there, :3774-3791), any shard when neither is known; accounts on
//    two shards: any shard as a surrogate (credit := debit fails accounts_must_be_different, one
//    check earlier and non-transient like the reference's status, which settle patches in).
//  * Imported events (execute_create :3066-3078, must_not_regress :3808-3817) are routed only
//    when the whole call is imported (flags[3]; each shard's slice is one batch), their timestamps
//    increase through the call and lie above every object of both grooves (the floor) and below
//    their own commit timestamps.
// The account directory's shard of two ids at once: both home slots load together, then both
// candidates' ids (the common case resolves at home: load <= 0.25); a miss continues the probe.
__device__ inline void dir_find2(const Dir& d, const tb_uint128_t& x, const tb_uint128_t& y,
                                 uint64_t* rx, uint64_t* ry) {
    const uint64_t sx = hash_id(x) & d.slots.mask, sy = hash_id(y) & d.slots.mask;
    const uint64_t wx = d.slots.slots[sx], wy = d.slots.slots[sy];
    const bool cx = slot_tag_is(wx, id_tag(x)), cy = slot_tag_is(wy, id_tag(y));
    const uint64_t qx = (wx & kRefMask) - 1, qy = (wy & kRefMask) - 1;
    tb_uint128_t ix{0, 0}, iy{0, 0};
    if (cx) ix = d.ids[qx];
    if (cy) iy = d.ids[qy];
    const tb_uint128_t* ids = d.ids;
    auto row_id = [=](uint64_t r) { return ids[r]; };
    // (probe_find_from returns a slot: its row is the slot word's ref)
    auto row_at = [&](uint64_t s) { return s == kNone ? kNone : (d.slots.slots[s] & kRefMask) - 1; };
    if (cx && u128_eq(ix, x)) *rx = qx;
    else if (wx == kEmpty) *rx = kNone;
    else *rx = row_at(probe_find_from(d.slots, x, probe_next(sx, d.slots.mask), row_id));
    if (cy && u128_eq(iy, y)) *ry = qy;
    else if (wy == kEmpty) *ry = kNone;
    else *ry = row_at(probe_find_from(d.slots, y, probe_next(sy, d.slots.mask), row_id));
}

// The id claim (device_common.hpp probe_claim) returning the slot and the ref it found there: the
// call's own (base + k + 1) when the claim took an empty slot, else the holder's -- no reload of
// the slot after the claim.
template <typename RowId>
__device__ inline uint64_t claim_ref(const IdTable& t, const tb_uint128_t& id, uint64_t ref,
                                     uint64_t row_base, RowId row_id, uint64_t* found) {
    const uint64_t tag = id_tag(id);
    const uint64_t tref = ref | tag;
    uint64_t s = hash_id(id) & t.mask;
    uint64_t w = t.slots[s];
    for (uint64_t n = 0; n < probe_limit(t.mask); n++) {
        if (w == kEmpty) {
            w = atomicCAS(&t.slots[s], (unsigned long long)kEmpty, (unsigned long long)tref);
            if (w == kEmpty) {
                *found = ref;
                return s;
            }
        }
        if (slot_tag_is(w, tag)) {
            const uint64_t r = (w & kRefMask) - 1;
            if (u128_eq(row_id(r), id)) {
                if (r >= row_base && tref < w) atomicMin(&t.slots[s], (unsigned long long)tref);
                *found = (w & kRefMask);
                return s;
            }
        }
        s = probe_next(s, t.mask);
        w = t.slots[s];
    }
    return kNone;
}

__global__ void __launch_bounds__(kRouteBlock) tbr_pass1(RouteArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_ev[kRouteBlock / 64][64 * kStageStride];
    const uint32_t k = blockIdx.x * kRouteBlock + threadIdx.x;
    const tb_transfer_t* mine = stage_wave_events(a.events, a.n, lds_ev[threadIdx.x >> 6]);
    bool hazard = false, pv_any = false, any = false;
    unsigned int kinds = 0;
    if (k < a.n) {
        const tb_transfer_t& t = *mine;
        const uint16_t f = t.flags;
        const bool post_void = (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
        const bool imported = (f & TB_TRANSFER_IMPORTED) != 0;
        uint8_t shard = kShardHazard, patch = 0;
        uint32_t slot = kNone32;
        const bool static_fail = (f & TB_TRANSFER_PADDING_MASK) != 0 ||
                                 (!imported && t.timestamp != 0) || u128_is_zero(t.id) ||
                                 u128_is_max(t.id);
        if (imported) {
            const uint32_t b = batch_of_guess(a.batch_ends, a.n_batches, a.n, k);
            const uint64_t stamp = a.batch_ts[b] - a.batch_ends[b] + k + 1;
            hazard = t.timestamp < TB_TIMESTAMP_MIN || t.timestamp >= stamp ||
                     t.timestamp <= a.imported_floor ||
                     (k > 0 && t.timestamp <= a.events[k - 1].timestamp);
        }
        kinds = imported ? 1u : 2u;
        if (!hazard && static_fail) {
            shard = kShardAny;
        } else if (!hazard) {
            const tb_transfer_t* ev = a.events;
            const tb_uint128_t* ids = a.tr.ids;
            const uint64_t base = a.base;
            // (the accounts' lookups are issued with the claim: neither waits on the other)
            uint64_t rd = kNone, rc = kNone;
            if (!post_void) dir_find2(a.acc, t.debit_account_id, t.credit_account_id, &rd, &rc);
            uint64_t found = 0;
            const uint64_t s = claim_ref(a.tr.slots, t.id, base + k + 1, base, [=](uint64_t r) {
                return r >= base ? ev[r - base].id : ids[r];
            }, &found);
            if (s == kNone) {
                set_flag(&a.flags[1], 1u);
                hazard = true;
            } else {
                slot = uint32_t(s);
                const uint64_t owner = found - 1;
                if (owner < base) {
                    shard = uint8_t(a.tr.shard[owner] & 0x7Fu);  // exists: decided on its holder
                } else if (post_void) {
                    shard = kShardPending;
                } else {
                    if (rd != kNone && rc != kNone && a.acc.shard[rd] != a.acc.shard[rc]) {
                        shard = kShardAny;
                        patch = cross_status(t);
                    } else if (rd != kNone) {
                        shard = a.acc.shard[rd];
                    } else if (rc != kNone) {
                        shard = a.acc.shard[rc];
                    } else {
                        shard = kShardAny;
                    }
                }
            }
        }
        any = shard == kShardAny;
        a.ev_shard[k] = hazard ? kShardHazard : shard;
        a.ev_slot[k] = slot;
        a.ev_patch[k] = patch;
        a.ev_keep[k] = 0;
        a.ev_link[k] = uint8_t(f & TB_TRANSFER_LINKED);
        a.tr.ids[a.base + k] = t.id;
        pv_any = post_void;
    }
    if (__any(pv_any) && (threadIdx.x & 63) == 0) set_flag(&a.flags[2], 1u);
    const uint64_t any_imported = __ballot(kinds & 1u), any_plain = __ballot(kinds & 2u);
    if ((threadIdx.x & 63) == 0 && (any_imported || any_plain))
        set_flag(&a.flags[3], (any_imported ? 1u : 0u) | (any_plain ? 2u : 0u));
    count_wave(&a.flags[4], any);
    raise_hazard(a, hazard);
}

// Pass 2, per post/void: the shard of its pending transfer -- the directory's holder, or the
// in-call event that creates it (post_or_void_pending_transfer reads only the pending transfer,
// its TransferPending status and its accounts, all on that shard, :4053-4299). A pending id found
// nowhere fails pending_transfer_not_found (:4100) after checks that read no state: any shard; so
// does one whose in-call creator fails whatever its shard (an event of any shard). A pending
// transfer created in the call by another post/void is a hazard.
// (A post/void of a pending transfer with a timeout resets pulse_next_timestamp on equality with
// the value over all shards, :4227-4229: the shards record their updates and the caller
// resolves them after the call -- tbg_pnt_ops.)
__global__ void __launch_bounds__(kRouteBlock) tbr_pass_pv(RouteArgs a) {
    const uint32_t k = blockIdx.x * kRouteBlock + threadIdx.x;
    bool hazard = false, any = false;
    if (k < a.n && a.ev_shard[k] == kShardPending) {
        const tb_transfer_t& t = a.events[k];
        const tb_transfer_t* ev = a.events;
        const tb_uint128_t* ids = a.tr.ids;
        const uint64_t base = a.base;
        const uint64_t s = probe_find(a.tr.slots, t.pending_id, [=](uint64_t r) {
            return r >= base ? ev[r - base].id : ids[r];
        });
        uint8_t shard = kShardAny;
        if (s != kNone) {
            const uint64_t r = (a.tr.slots.slots[s] & kRefMask) - 1;
            if (r < base) {
                shard = a.tr.shard[r] & 0x7Fu;
            } else {
                const tb_transfer_t& p = ev[r - base];
                const bool p_pv = (p.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
                const uint8_t ps = a.ev_shard[r - base];
                shard = p_pv || ps == kShardHazard ? kShardHazard : ps;
            }
        }
        hazard = shard == kShardHazard;
        any = shard == kShardAny;
        a.ev_shard[k] = shard;
    }
    count_wave(&a.flags[4], any);
    raise_hazard(a, hazard);
}

// Pass 3, per event whose id repeats an earlier event's of the call (the slot's final owner, the
// serial order's first occurrence): it runs on the first occurrence's shard -- created or orphaned
// there, the repeat is decided by create_transfer_exists / id_already_failed on that shard;
// failed otherwise, the repeat executes afresh, which it may do there when its own placement is
// any shard or the same. Else, or when the first occurrence runs anywhere, or the repeat is a
// surrogate (whose exists comparison would see its substituted account), a hazard.
__global__ void __launch_bounds__(kRouteBlock) tbr_pass_dup(RouteArgs a) {
    const uint32_t k = blockIdx.x * kRouteBlock + threadIdx.x;
    bool hazard = false, repeat = false;
    uint32_t owner = kNone32;
    if (k < a.n && a.ev_slot[k] != kNone32 && a.ev_shard[k] != kShardHazard) {
        const uint64_t r = (a.tr.slots.slots[a.ev_slot[k]] & kRefMask) - 1;
        if (r >= a.base && r != a.base + k) {
            repeat = true;
            owner = uint32_t(r - a.base);
            const uint8_t own = a.ev_shard[k];
            const uint8_t first = a.ev_shard[r - a.base];
            const bool ok = a.ev_patch[k] == 0 && first < kShardAny &&
                            (own == kShardAny || own == first);
            a.ev_shard[k] = ok ? first : kShardHazard;
            hazard = !ok;
        }
    }
    if (k < a.n) a.ev_owner[k] = owner;
    count_wave(&a.flags[6], repeat);
    raise_hazard(a, hazard);
}

// Pass 4, per chain head: linked chains (:3002-3213) are atomic, so a chain goes to a shard whole
// -- every event pinned to the same shard, the chain's events that may run anywhere with them --
// and a chain left open at its batch's end (the slice is one batch on its shard) is a hazard.
// A single event that may run anywhere goes to shard k mod shards.
__global__ void __launch_bounds__(kRouteBlock) tbr_pass_chains(RouteArgs a) {
    const uint32_t k = blockIdx.x * kRouteBlock + threadIdx.x;
    bool hazard = false;
    if (k < a.n) {
        const uint32_t b = batch_of_guess(a.batch_ends, a.n_batches, a.n, k);
        const uint32_t bstart = b ? a.batch_ends[b - 1] : 0, bend = a.batch_ends[b];
        const bool head = k == bstart || !a.ev_link[k - 1];
        const bool linked = a.ev_link[k] != 0;
        if (head && !linked) {
            if (a.ev_shard[k] == kShardAny) a.ev_shard[k] = uint8_t(k % a.shards);
        } else if (head) {
            uint32_t sh = kShardAny, j = k;
            bool closed = false;
            for (; j < bend; j++) {
                const uint8_t c = a.ev_shard[j];
                if (c >= kShardPending || (c < kShardAny && sh != kShardAny && c != sh)) {
                    hazard = true;
                    break;
                }
                if (c < kShardAny) sh = c;
                if (!a.ev_link[j]) {
                    closed = true;
                    break;
                }
            }
            hazard = hazard || !closed;
            if (!hazard) {
                if (sh == kShardAny) sh = uint8_t(k % a.shards);
                for (uint32_t x = k; x <= j; x++) a.ev_shard[x] = uint8_t(sh);
            }
        }
    }
    raise_hazard(a, hazard);
}

// Per-block counts per shard of the scatter (every event placed by now, else a hazard).
__global__ void __launch_bounds__(kRouteBlock) tbr_pass_count(RouteArgs a) {
    __shared__ unsigned int cnt[kShardsMax];
    for (uint32_t s = threadIdx.x; s < a.shards; s += kRouteBlock) cnt[s] = 0;
    __syncthreads();
    const uint32_t k = blockIdx.x * kRouteBlock + threadIdx.x;
    bool hazard = false, patched = false;
    if (k < a.n) {
        const uint8_t sh = a.ev_shard[k];
        hazard = sh >= a.shards;
        patched = a.ev_patch[k] != 0;
        if (!hazard) atomicAdd(&cnt[sh], 1u);
    }
    count_wave(&a.flags[5], patched);
    raise_hazard(a, hazard);
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < a.shards; s += kRouteBlock)
        a.block_counts[uint64_t(s) * a.nblocks + blockIdx.x] = cnt[s];
}

// Shard-major offsets of the scatter: workgroup s scans row s of the per-block counts (exclusive,
// row-local; wave shuffles, one barrier pair per 1,024 counts) and writes the row's total -- the
// host reads W totals, not W x blocks counts.
constexpr uint32_t kScanThreads = 1024;
__global__ void __launch_bounds__(kScanThreads) tbr_scan_counts(const uint32_t* counts,
                                                                uint32_t nblocks,
                                                                uint32_t* offsets,
                                                                uint32_t* totals) {
    __shared__ uint32_t wave_sum[kScanThreads / 64];
    const uint32_t s = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t* row = counts + uint64_t(s) * nblocks;
    uint32_t* out = offsets + uint64_t(s) * nblocks;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += kScanThreads) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t v = b < nblocks ? row[b] : 0;
        uint32_t x = v;  // inclusive scan within the wave
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane == 63) wave_sum[wv] = x;
        __syncthreads();
        uint32_t before = carry, total = 0;
        for (uint32_t w = 0; w < kScanThreads / 64; w++) {
            const uint32_t t = wave_sum[w];
            if (w < wv) before += t;
            total += t;
        }
        if (b < nblocks) out[b] = before + x - v;
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[s] = carry;
}

// A call with a hazard takes nothing: its claims are released.
__global__ void tbr_release(RouteArgs a) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n) return;
    const uint32_t s = a.ev_slot[k];
    if (s == kNone32) return;
    unsigned long long* w = &a.tr.slots.slots[s];
    if ((*w & kRefMask) == a.base + k + 1) *w = kTomb;
}

// Each event copied to its shard's slice with its global commit timestamp and its position (a
// surrogate with its credit account replaced by its debit account); its shard into the store.
// The wave's events are staged in LDS with coalesced loads (stage_wave_events), and each 8-lane
// group then stores one event's 128 contiguous bytes to its slot in its shard's slice: a wave's
// events bound for one shard land in consecutive slots, so the stores (across xGMI for another
// GPU's slice) are as coalesced as the loads. (A lane copying its own event issued 8 loads and 8
// stores that each touched 64 lines.)
__global__ void __launch_bounds__(kRouteBlock) tbr_pass2(RouteArgs a, const uint32_t* offsets,
                                                         const SliceDst* dst_tab,
                                                         uint32_t* out_pos) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_ev[kRouteBlock / 64][64 * kStageStride];
    __shared__ unsigned long long lds_dst[kRouteBlock / 64][64];
    __shared__ unsigned int wave_cnt[kRouteBlock / 64][kShardsMax];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t k = blockIdx.x * kRouteBlock + threadIdx.x;
    const bool active = k < a.n;
    const uint32_t s = active ? a.ev_shard[k] : 0xFFu;
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t my_rank = 0;
    for (uint32_t sv = 0; sv < a.shards; sv++) {
        const uint64_t m = __ballot(active && s == sv);
        if (lane == 0) wave_cnt[wv][sv] = __popcll(m);
        if (s == sv) my_rank = __popcll(m & lt);
    }
    const uint8_t* my = lds_ev[wv];
    stage_wave_events(a.events, a.n, lds_ev[wv]);
    __syncthreads();
    // this lane's event: its slot (bit 0: a surrogate -- credit_account_id := debit_account_id)
    unsigned long long dst = 0;
    if (active) {
        uint32_t rank = my_rank;
        for (uint32_t w = 0; w < wv; w++) rank += wave_cnt[w][s];
        const SliceDst d = dst_tab[s];
        const uint32_t pos = offsets[uint64_t(s) * a.nblocks + blockIdx.x] + rank;
        dst = reinterpret_cast<unsigned long long>(&d.events[pos]) | (a.ev_patch[k] ? 1ull : 0ull);
        const uint32_t b = batch_of_guess(a.batch_ends, a.n_batches, a.n, k);
        d.timestamps[pos] = a.batch_ts[b] - a.batch_ends[b] + k + 1;
        out_pos[d.base + pos] = k;
        a.tr.shard[a.base + k] = uint8_t(s);
    }
    lds_dst[wv][lane] = dst;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const uint32_t part = lane & 7;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t e = i * 8 + (lane >> 3);
        const unsigned long long de = lds_dst[wv][e];
        if (de == 0) continue;
        // (a surrogate's part 2, bytes 32..47, is its part 1: credit := debit)
        const uint32_t src_part = (part == 2 && (de & 1ull)) ? 1u : part;
        const v4u v = *reinterpret_cast<const v4u*>(
            __builtin_assume_aligned(my + e * kStageStride + src_part * 16, 16));
        *reinterpret_cast<v4u*>((de & ~1ull) + part * 16) = v;
    }
}

// Results back to call order, a surrogate's status patched to the reference's; an id that now
// exists on its shard (created, or orphaned by a transient failure) by any of its occurrences
// keeps its slot (ev_keep of the first occurrence, whose store row holds the id and the shard).
// The largest timestamp of a created transfer goes to key_max (the transfers objects tree's
// key_range.key_max, which the imported floor follows): a maximum per workgroup in block_max,
// reduced by tbr_settle_release's first workgroup.
__global__ void __launch_bounds__(kRouteBlock) tbr_settle(RouteArgs a, const SliceDst* dst_tab,
                                                          const uint32_t* pos,
                                                          tb_create_result_t* results,
                                                          unsigned long long* block_max) {
    __shared__ uint64_t wave_max[kRouteBlock / 64];
    __shared__ uint32_t bases[kShardsMax + 1];
    for (uint32_t s = threadIdx.x; s < a.shards; s += kRouteBlock) bases[s] = dst_tab[s].base;
    if (threadIdx.x == 0) bases[a.shards] = a.n;
    __syncthreads();
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t ts_max = 0;
    if (j < a.n) {
        uint32_t s = 0;  // (the shard whose slice holds position j: bases ascend)
        while (bases[s + 1] <= j) s++;
        const uint32_t k = pos[j];
        // (the results may live in the shard's GPU: read across xGMI)
        tb_create_result_t r = dst_tab[s].results[j - bases[s]];
        if (a.ev_patch[k] && r.status == TB_CT_ACCOUNTS_MUST_BE_DIFFERENT) r.status = a.ev_patch[k];
        results[k] = r;
        const bool created = r.status == TB_STATUS_CREATED;
        if (created) ts_max = r.timestamp;
        if ((created || tb_transfer_status_transient(r.status)) && a.ev_slot[k] != kNone32) {
            const uint32_t o = a.ev_owner[k];
            a.ev_keep[o == kNone32 ? k : o] = 1;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t other = __shfl_xor(ts_max, off);
        ts_max = other > ts_max ? other : ts_max;
    }
    if ((threadIdx.x & 63) == 0) wave_max[threadIdx.x >> 6] = ts_max;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t m = 0;
        for (uint32_t w = 0; w < kRouteBlock / 64; w++) m = wave_max[w] > m ? wave_max[w] : m;
        block_max[blockIdx.x] = m;
    }
}

// ... then the slots of first occurrences whose id exists nowhere are released; the first
// workgroup reduces the per-workgroup maxima to key_max.
__global__ void __launch_bounds__(kRouteBlock) tbr_settle_release(
    RouteArgs a, const unsigned long long* block_max, uint32_t nblocks,
    unsigned long long* key_max) {
    if (blockIdx.x == 0) {
        __shared__ uint64_t part[kRouteBlock];
        uint64_t m = 0;
        for (uint32_t b = threadIdx.x; b < nblocks; b += kRouteBlock)
            m = block_max[b] > m ? block_max[b] : m;
        part[threadIdx.x] = m;
        __syncthreads();
        for (uint32_t w = kRouteBlock / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w && part[threadIdx.x + w] > part[threadIdx.x])
                part[threadIdx.x] = part[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) *key_max = part[0];
    }
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n) return;
    const uint32_t s = a.ev_slot[k];
    if (s == kNone32 || a.ev_keep[k] || a.ev_owner[k] != kNone32) return;
    // (a first occurrence's own claim -- not the slot of an id that already existed)
    unsigned long long* w = &a.tr.slots.slots[s];
    if ((*w & kRefMask) == a.base + k + 1) *w = kTomb;
}

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace

struct tbr_ctx {
    uint32_t shards = 0, events_max = 0;
    hipStream_t stream = nullptr;
    Dir acc{}, tr{};
    uint64_t acc_used = 0, acc_cap = 0, tr_used = 0, tr_cap = 0;
    uint8_t* ev_shard = nullptr;
    uint32_t* ev_slot = nullptr;
    uint8_t* ev_patch = nullptr;
    uint8_t* ev_keep = nullptr;
    uint8_t* ev_link = nullptr;
    uint32_t* ev_owner = nullptr;
    uint64_t route_stats[3] = {0, 0, 0};  // the last routed call's (anywhere, surrogates, repeats)
    uint32_t* block_counts = nullptr;
    uint32_t* offsets = nullptr;
    unsigned int* flags = nullptr;
    unsigned long long* key_max = nullptr;  // settle: created timestamps' maximum
    unsigned long long* block_max = nullptr;  // ... per settle workgroup
    uint32_t* totals = nullptr;               // per shard: the routed call's events
    SliceDst* d_tab = nullptr;                // the routed call's slices (device copy of tab)
    std::vector<SliceDst> tab;
    uint64_t imported_floor = ~0ull;        // tbr_set_imported_floor (none yet: every import)
    tb_uint128_t* q_ids = nullptr;  // lookup / record staging (events_max)
    int32_t* q_out = nullptr;
    // the routed call awaiting tbr_settle_device
    bool pending = false;
    uint64_t call_base = 0;
    uint32_t call_n = 0;
};

namespace {

template <typename T>
bool alloc(T** p, uint64_t count, bool zero, hipStream_t s) {
    if (hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(count * sizeof(T), 16)) !=
        hipSuccess)
        return false;
    return !zero || hipMemsetAsync(*p, 0, std::max<size_t>(count * sizeof(T), 16), s) == hipSuccess;
}

RouteArgs route_args(tbr_ctx* r, const tb_transfer_t* ev, uint32_t n, const uint32_t* ends,
                     const uint64_t* bts, uint32_t nb) {
    RouteArgs a{};
    a.acc = r->acc;
    a.tr = r->tr;
    a.events = ev;
    a.n = n;
    a.batch_ends = ends;
    a.batch_ts = bts;
    a.n_batches = nb;
    a.base = r->tr_used;
    a.shards = r->shards;
    a.nblocks = (n + kRouteBlock - 1) / kRouteBlock;
    a.ev_shard = r->ev_shard;
    a.ev_slot = r->ev_slot;
    a.ev_patch = r->ev_patch;
    a.ev_keep = r->ev_keep;
    a.ev_link = r->ev_link;
    a.ev_owner = r->ev_owner;
    a.block_counts = r->block_counts;
    a.flags = r->flags;
    a.imported_floor = r->imported_floor;
    return a;
}

int record(tbr_ctx* r, Dir& d, uint64_t& used, uint64_t cap, const tb_uint128_t* ids,
           const uint8_t* shards, uint32_t n) {
    if (n == 0) return 0;
    if (used + n > cap) return -28;
    if (hipMemcpyAsync(d.ids + used, ids, size_t(n) * 16, hipMemcpyHostToDevice, r->stream) ||
        hipMemcpyAsync(d.shard + used, shards, n, hipMemcpyHostToDevice, r->stream) ||
        hipMemsetAsync(r->flags, 0, 8, r->stream))
        return -5;
    hipLaunchKernelGGL(tbr_insert, dim3((n + 255) / 256), dim3(256), 0, r->stream, d, used, n,
                       r->flags);
    unsigned int f[2] = {0, 0};
    if (hipMemcpyAsync(f, r->flags, 8, hipMemcpyDeviceToHost, r->stream) ||
        hipStreamSynchronize(r->stream))
        return -5;
    used += n;
    return f[1] ? -28 : 0;
}

int64_t lookup(tbr_ctx* r, const Dir& d, const tb_uint128_t* ids, uint32_t n, int32_t* out) {
    for (uint32_t a = 0; a < n; a += r->events_max) {
        const uint32_t m = std::min(n - a, r->events_max);
        if (hipMemcpyAsync(r->q_ids, ids + a, size_t(m) * 16, hipMemcpyHostToDevice, r->stream))
            return -5;
        hipLaunchKernelGGL(tbr_lookup, dim3((m + 255) / 256), dim3(256), 0, r->stream, d, r->q_ids,
                           m, r->q_out);
        if (hipMemcpyAsync(out + a, r->q_out, size_t(m) * 4, hipMemcpyDeviceToHost, r->stream) ||
            hipStreamSynchronize(r->stream))
            return -5;
    }
    return n;
}

}  // namespace

namespace {

// The device path of one call (tbr_route_device / _slices): the placement passes, the offsets
// scanned on the device (the host reads the W totals with the flags: one synchronisation), the
// slice table (a shard's events / timestamps at `slices`, or contiguous in shard order at c_ev /
// c_ts) uploaded, the scatter.
int64_t route_impl(tbr_ctx* r, const tb_transfer_t* d_events, uint32_t n,
                   const uint32_t* d_batch_ends, const uint64_t* d_batch_ts, uint32_t n_batches,
                   const tbr_slice* slices, tb_transfer_t* c_ev, uint64_t* c_ts,
                   uint32_t* d_out_pos, uint32_t* shard_counts) {
    if (!r || r->pending || n > r->events_max || n_batches == 0) return -22;
    if (r->tr_used + n > r->tr_cap) return -28;
    RouteArgs a = route_args(r, d_events, n, d_batch_ends, d_batch_ts, n_batches);
    const dim3 grid(a.nblocks), block(kRouteBlock);
    const uint32_t W = r->shards;
    if (hipMemsetAsync(r->flags, 0, 32, r->stream)) return -5;
    hipLaunchKernelGGL(tbr_pass1, grid, block, 0, r->stream, a);
    hipLaunchKernelGGL(tbr_pass_pv, grid, block, 0, r->stream, a);
    hipLaunchKernelGGL(tbr_pass_dup, grid, block, 0, r->stream, a);
    hipLaunchKernelGGL(tbr_pass_chains, grid, block, 0, r->stream, a);
    hipLaunchKernelGGL(tbr_pass_count, grid, block, 0, r->stream, a);
    hipLaunchKernelGGL(tbr_scan_counts, dim3(W), dim3(kScanThreads), 0, r->stream,
                       r->block_counts, a.nblocks, r->offsets, r->totals);
    unsigned int f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<uint32_t> totals(W);
    if (hipMemcpyAsync(f, r->flags, 32, hipMemcpyDeviceToHost, r->stream) ||
        hipMemcpyAsync(totals.data(), r->totals, size_t(W) * 4, hipMemcpyDeviceToHost,
                       r->stream) ||
        hipStreamSynchronize(r->stream))
        return -5;
    if (f[3] == 3u) f[0] = 1;  // imported and non-imported events in one call
    r->route_stats[0] = f[4];
    r->route_stats[1] = f[5];
    r->route_stats[2] = f[6];
    bool over = false;  // (a slice too small for its part: nothing is scattered)
    for (uint32_t s = 0; s < W && slices; s++) over |= totals[s] > slices[s].capacity;
    if (f[0] || f[1] || over) {
        hipLaunchKernelGGL(tbr_release, grid, block, 0, r->stream, a);
        if (hipStreamSynchronize(r->stream)) return -5;
        return f[1] ? -28 : (over && !f[0]) ? -22 : 1;
    }
    uint64_t base = 0;
    for (uint32_t s = 0; s < W; s++) {
        SliceDst& d = r->tab[s];
        d.base = base;
        if (slices) {
            d.events = slices[s].events;
            d.timestamps = slices[s].timestamps;
            d.results = slices[s].results;
        } else {
            d.events = c_ev + base;
            d.timestamps = c_ts + base;
            d.results = nullptr;  // (tbr_settle_device's d_shard_results)
        }
        shard_counts[s] = totals[s];
        base += totals[s];
    }
    if (hipMemcpyAsync(r->d_tab, r->tab.data(), sizeof(SliceDst) * W, hipMemcpyHostToDevice,
                       r->stream))
        return -5;
    hipLaunchKernelGGL(tbr_pass2, grid, block, 0, r->stream, a, r->offsets, r->d_tab, d_out_pos);
    if (hipGetLastError() || hipStreamSynchronize(r->stream)) return -5;
    r->pending = true;
    r->call_base = a.base;
    r->call_n = n;
    return f[2] ? 2 : 0;
}

}  // namespace

extern "C" {

tbr_ctx* tbr_open(uint32_t shards, uint64_t account_capacity, uint64_t transfer_capacity,
                  uint32_t events_max, uint32_t device) {
    if (shards == 0 || shards > kShardsMax || events_max == 0 ||
        account_capacity >= (1ull << 31) || transfer_capacity >= (1ull << 31))
        return nullptr;
    if (hipSetDevice(int(device)) != hipSuccess) return nullptr;
    tbr_ctx* r = new tbr_ctx();
    r->shards = shards;
    r->events_max = events_max;
    r->tab.assign(shards, SliceDst{nullptr, nullptr, nullptr, 0});
    r->acc_cap = account_capacity;
    r->tr_cap = transfer_capacity;
    const uint64_t acc_slots = std::max<uint64_t>(next_pow2(account_capacity * 4), 64);
    const uint64_t tr_slots = std::max<uint64_t>(next_pow2(transfer_capacity * 4), 64);
    const uint32_t nblocks = (events_max + kRouteBlock - 1) / kRouteBlock;
    bool ok = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && alloc(&r->acc.slots.slots, acc_slots, true, r->stream) &&
         alloc(&r->acc.ids, account_capacity, false, r->stream) &&
         alloc(&r->acc.shard, account_capacity, false, r->stream) &&
         alloc(&r->tr.slots.slots, tr_slots, true, r->stream) &&
         alloc(&r->tr.ids, transfer_capacity, true, r->stream) &&
         alloc(&r->tr.shard, transfer_capacity, true, r->stream) &&
         alloc(&r->ev_shard, events_max, false, r->stream) &&
         alloc(&r->ev_slot, events_max, false, r->stream) &&
         alloc(&r->ev_patch, events_max, false, r->stream) &&
         alloc(&r->ev_keep, events_max, false, r->stream) &&
         alloc(&r->ev_link, events_max, false, r->stream) &&
         alloc(&r->ev_owner, events_max, false, r->stream) &&
         alloc(&r->block_counts, uint64_t(shards) * nblocks, false, r->stream) &&
         alloc(&r->offsets, uint64_t(shards) * nblocks, false, r->stream) &&
         alloc(&r->flags, 8, true, r->stream) && alloc(&r->key_max, 1, true, r->stream) &&
         alloc(&r->block_max, nblocks, true, r->stream) &&
         alloc(&r->totals, shards, true, r->stream) && alloc(&r->d_tab, shards, true, r->stream) &&
         alloc(&r->q_ids, events_max, false, r->stream) &&
         alloc(&r->q_out, events_max, false, r->stream);
    ok = ok && hipStreamSynchronize(r->stream) == hipSuccess;
    if (!ok) {
        fprintf(stderr, "tbr_open: allocation failed\n");
        tbr_close(r);
        return nullptr;
    }
    r->acc.slots.mask = acc_slots - 1;
    r->tr.slots.mask = tr_slots - 1;
    return r;
}

void tbr_close(tbr_ctx* r) {
    if (!r) return;
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    void* ptrs[] = {r->acc.slots.slots, r->acc.ids, r->acc.shard, r->tr.slots.slots, r->tr.ids,
                    r->tr.shard, r->ev_shard, r->ev_slot, r->ev_patch, r->ev_keep, r->ev_link, r->ev_owner, r->block_counts, r->offsets, r->flags,
                    r->key_max, r->block_max, r->totals, r->d_tab, r->q_ids, r->q_out};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
}

int tbr_record_accounts(tbr_ctx* r, const tb_uint128_t* ids, const uint8_t* shards, uint32_t n) {
    if (!r || r->pending) return -22;
    return record(r, r->acc, r->acc_used, r->acc_cap, ids, shards, n);
}

int tbr_record_transfers(tbr_ctx* r, const tb_uint128_t* ids, const uint8_t* shards, uint32_t n) {
    if (!r || r->pending) return -22;
    return record(r, r->tr, r->tr_used, r->tr_cap, ids, shards, n);
}

int64_t tbr_account_shards(tbr_ctx* r, const tb_uint128_t* ids, uint32_t n, int32_t* out) {
    if (!r) return -22;
    return lookup(r, r->acc, ids, n, out);
}

int64_t tbr_transfer_shards(tbr_ctx* r, const tb_uint128_t* ids, uint32_t n, int32_t* out) {
    if (!r) return -22;
    return lookup(r, r->tr, ids, n, out);
}

int64_t tbr_route_device(tbr_ctx* r, const tb_transfer_t* d_events, uint32_t n,
                         const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                         uint32_t n_batches, tb_transfer_t* d_out_events, uint64_t* d_out_ts,
                         uint32_t* d_out_pos, uint32_t* shard_counts) {
    return route_impl(r, d_events, n, d_batch_ends, d_batch_ts, n_batches, nullptr, d_out_events,
                      d_out_ts, d_out_pos, shard_counts);
}

int64_t tbr_route_device_slices(tbr_ctx* r, const tb_transfer_t* d_events, uint32_t n,
                                const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                                uint32_t n_batches, const tbr_slice* slices,
                                uint32_t* d_out_pos, uint32_t* shard_counts) {
    if (!slices) return -22;
    return route_impl(r, d_events, n, d_batch_ends, d_batch_ts, n_batches, slices, nullptr,
                      nullptr, d_out_pos, shard_counts);
}

int tbr_route_stats(tbr_ctx* r, uint64_t* out) {
    if (!r || !out) return -22;
    for (int i = 0; i < 3; i++) out[i] = r->route_stats[i];
    return 0;
}

int tbr_set_imported_floor(tbr_ctx* r, uint64_t floor) {
    if (!r) return -22;
    r->imported_floor = floor;
    return 0;
}

int tbr_settle_device(tbr_ctx* r, const tb_create_result_t* d_shard_results,
                      const uint32_t* d_positions, uint32_t n, tb_create_result_t* d_results,
                      uint64_t* created_timestamp_max) {
    if (!r || !r->pending || n != r->call_n) return -22;
    RouteArgs a = route_args(r, nullptr, n, nullptr, nullptr, 1);
    a.base = r->call_base;
    unsigned long long km = 0;
    const uint32_t nb = (n + kRouteBlock - 1) / kRouteBlock;
    if (d_shard_results) {  // (contiguous results in shard order, else the routed slices')
        for (uint32_t s = 0; s < r->shards; s++) r->tab[s].results = d_shard_results + r->tab[s].base;
        if (hipMemcpyAsync(r->d_tab, r->tab.data(), sizeof(SliceDst) * r->shards,
                           hipMemcpyHostToDevice, r->stream))
            return -5;
    }
    for (uint32_t s = 0; s < r->shards; s++)
        if (!r->tab[s].results && r->tab[s].base < (s + 1 < r->shards ? r->tab[s + 1].base : n))
            return -22;
    hipLaunchKernelGGL(tbr_settle, dim3(nb), dim3(kRouteBlock), 0, r->stream, a, r->d_tab,
                       d_positions, d_results, r->block_max);
    hipLaunchKernelGGL(tbr_settle_release, dim3(nb), dim3(kRouteBlock), 0, r->stream, a,
                       r->block_max, nb, r->key_max);
    if (hipGetLastError() || hipMemcpyAsync(&km, r->key_max, 8, hipMemcpyDeviceToHost, r->stream) ||
        hipStreamSynchronize(r->stream))
        return -5;
    if (created_timestamp_max) *created_timestamp_max = km;
    r->tr_used = r->call_base + n;
    r->pending = false;
    return 0;
}

}  // extern "C"
