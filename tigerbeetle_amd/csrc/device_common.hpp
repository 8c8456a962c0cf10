// Device-side building blocks of the executor: u128 helpers, the HBM id tables, slot encoding.
//
// Tables (one per groove of the reference's Forest, src/state_machine.zig:278-283):
//   * rows: an append-only array of 128-byte objects (tb_account_t / tb_transfer_t). Row r of
//     the transfer store is the r-th create_transfers event ever submitted (likewise accounts), so
//     an in-flight event and its row share one index; `live[r]` says whether row r is an object.
//   * slots: an open-addressing (linear probing) hash index id -> row, one u64 word per slot:
//       0                 empty
//       kTomb             deleted (a claim whose event did not create an object); probes skip it
//       tag | (row + 1)   the object at `row`: bits 0-31 row + 1, bits 32-61 a 30-bit tag of the
//                         id (a probe passes a slot whose tag differs without reading its row),
//                         bit 62 set: an orphaned id (transfers only)
//     During a call, a slot may hold an in-flight claim: tag | (row + 1) with row >= row_base of
//     the call; the id of such a row is read from the call's input events. Claims race with
//     atomicCAS(0 -> ref) and duplicates resolve with atomicMin, so the earliest event of the call
//     owns the slot -- the serial order's first occurrence.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tb_types.h"

namespace tbg {

typedef unsigned __int128 u128;

constexpr uint64_t kEmpty = 0;
constexpr uint64_t kTomb = ~0ull;
constexpr uint64_t kOrphanBit = 1ull << 62;
constexpr uint64_t kRefMask = 0xFFFFFFFFull;            // row + 1
constexpr uint64_t kTagMask = ((1ull << 30) - 1) << 32;
constexpr uint64_t kNone = ~0ull;  // "no row" in per-event scratch
constexpr u128 kU128Max = ~(u128)0;

__host__ __device__ inline u128 U(const tb_uint128_t& x) { return ((u128)x.hi << 64) | x.lo; }
__host__ __device__ inline tb_uint128_t W(u128 x) {
    tb_uint128_t r;
    r.lo = (uint64_t)x;
    r.hi = (uint64_t)(x >> 64);
    return r;
}
// sum_overflows (state_machine.zig:5144-5149): whether a + b overflows Int (std.math.add's
// error), for the u64 and u128 widths the reference instantiates (:5163-5166).
template <typename Int>
__host__ __device__ inline bool sum_overflows(Int a, Int b) {
    return Int(a + b) < a;
}
__host__ __device__ inline bool u128_eq(const tb_uint128_t& a, const tb_uint128_t& b) {
    return a.lo == b.lo && a.hi == b.hi;
}
__host__ __device__ inline bool u128_is_zero(const tb_uint128_t& a) { return (a.lo | a.hi) == 0; }
__host__ __device__ inline bool u128_is_max(const tb_uint128_t& a) {
    return (a.lo & a.hi) == ~0ull;
}

__host__ __device__ inline uint64_t mix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h;
}
// Home slot of an id, and the probe sequence. Ids that differ only in their 4 low bits share one
// 16-slot group (one 128-byte line): sequential ids (the reference's --id-order=sequential, and
// TigerBeetle's recommended time-based ids within a millisecond) land in one line per 16 ids, so a
// wave's claims touch 4-5 lines instead of 64. The offset inside the group is the id's low bits
// XOR bits of the group hash, so ids that share their low bits (strided ids) still spread over
// every offset. A probe steps a whole group at a time (s + 16): an id whose home group is taken
// by another run of sequential ids reaches a free group in one step instead of walking the run.
constexpr uint64_t kProbeStride = 16;

__host__ __device__ inline uint64_t hash_id(const tb_uint128_t& id) {
    const uint64_t group = mix64((id.lo >> 4) ^ mix64(id.hi + 0x9E3779B97F4A7C15ull));
    return (group << 4) | ((id.lo ^ (group >> 59)) & 15);
}
__host__ __device__ inline uint64_t probe_next(uint64_t s, uint64_t mask) {
    return (s + kProbeStride) & mask;
}
// Slots a probe may visit before it has seen every slot of its offset class once.
__host__ __device__ inline uint64_t probe_limit(uint64_t mask) { return (mask >> 4) + 1; }

// The id's tag in slot-word position (independent of the home slot's bits).
__host__ __device__ inline uint64_t id_tag(const tb_uint128_t& id) {
    return (mix64(id.hi ^ mix64(id.lo ^ 0x2545F4914F6CDD1Dull)) >> 34) << 32;
}
// A live slot word (not empty, not a tombstone) whose tag is `tag`.
__host__ __device__ inline bool slot_tag_is(uint64_t w, uint64_t tag) {
    return w != kEmpty && w != kTomb && (w & kTagMask) == tag;
}

// Non-temporal / plain 16-byte vector copies of 128-byte rows.
struct alignas(16) Row128 {
    uint4 q[8];
};

__device__ inline void copy_row(void* dst, const void* src) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = s[i];
}

// u128 atomic add/sub on a {lo, hi} pair: the carry/borrow of each u64 add is propagated with a
// second atomic. Concurrent adds commute, so the final value is the exact sum.
// atomic_add_u128 returns the hi word it produced when it changed the hi word (else 0): the
// adder that moves the hi word last observes its final value.
__device__ inline uint64_t atomic_add_u128(tb_uint128_t* p, u128 v) {
    uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    if (lo) {
        uint64_t old = atomicAdd((unsigned long long*)&p->lo, (unsigned long long)lo);
        if (old + lo < old) hi += 1;
    }
    if (hi) return atomicAdd((unsigned long long*)&p->hi, (unsigned long long)hi) + hi;
    return 0;
}
__device__ inline void atomic_sub_u128(tb_uint128_t* p, u128 v) {
    uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    if (lo) {
        uint64_t old = atomicAdd((unsigned long long*)&p->lo, (unsigned long long)(0 - lo));
        if (old < lo) hi += 1;  // borrow
    }
    if (hi) atomicAdd((unsigned long long*)&p->hi, (unsigned long long)(0 - hi));
}

// The 32-bit word holding {code, flags} of an Account (offset 116): flags are its high half.
__device__ inline uint32_t* account_code_flags_word(tb_account_t* a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a) + 116);
}

// A table view passed by value to kernels.
struct IdTable {
    unsigned long long* slots;
    uint64_t mask;  // slot count - 1
};

// Read-only probe: returns the slot index holding `id`, or kNone. `row_id(r)` gives the id of row
// r (committed rows from the store, in-flight rows from the call's input).
template <typename RowId>
__device__ inline uint64_t probe_find_from(const IdTable& t, const tb_uint128_t& id, uint64_t s,
                                           RowId row_id) {
    const uint64_t tag = id_tag(id);
    for (uint64_t n = 0; n < probe_limit(t.mask); n++) {
        uint64_t w = t.slots[s];
        if (w == kEmpty) return kNone;
        if (slot_tag_is(w, tag)) {
            uint64_t r = (w & kRefMask) - 1;
            if (u128_eq(row_id(r), id)) return s;
        }
        s = probe_next(s, t.mask);
    }
    return kNone;
}
template <typename RowId>
__device__ inline uint64_t probe_find(const IdTable& t, const tb_uint128_t& id, RowId row_id) {
    return probe_find_from(t, id, hash_id(id) & t.mask, row_id);
}

// Claim-or-find: inserts an in-flight claim `ref` for `id` unless `id` is already present.
// Returns the slot of `id`. Duplicates within the call keep the smallest ref (earliest event).
// `*dup` is set when another in-flight claim of the same id is found: of two same-id events, the
// one probing second always sees the other's claim, so a call with no `dup` has unique ids.
// `s` is the slot to start at and `w` its word as already read (the home slot, normally).
template <typename RowId>
__device__ inline uint64_t probe_claim_from(const IdTable& t, const tb_uint128_t& id, uint64_t ref,
                                            uint64_t row_base, RowId row_id, bool* dup,
                                            uint64_t s, uint64_t w) {
    const uint64_t tag = id_tag(id);
    const uint64_t tref = ref | tag;
    for (uint64_t n = 0; n < probe_limit(t.mask); n++) {
        if (w == kEmpty) {
            w = atomicCAS(&t.slots[s], (unsigned long long)kEmpty, (unsigned long long)tref);
            if (w == kEmpty) return s;
        }
        if (slot_tag_is(w, tag)) {
            uint64_t r = (w & kRefMask) - 1;
            if (u128_eq(row_id(r), id)) {
                if (r >= row_base) {
                    *dup = true;
                    if (tref < w) atomicMin(&t.slots[s], (unsigned long long)tref);
                }
                return s;
            }
        }
        s = probe_next(s, t.mask);
        w = t.slots[s];
    }
    return kNone;  // table full: the host sizes tables so this cannot happen
}
template <typename RowId>
__device__ inline uint64_t probe_claim(const IdTable& t, const tb_uint128_t& id, uint64_t ref,
                                       uint64_t row_base, RowId row_id, bool* dup) {
    const uint64_t s = hash_id(id) & t.mask;
    return probe_claim_from(t, id, ref, row_base, row_id, dup, s, t.slots[s]);
}

// The account index: a read-mostly cache of the id -> row mapping together with what the
// create_transfers checks read of an account, in 16-byte entries carrying the id's low word, the
// row, the static flags, the hazard bits and the ledger's low 16 bits: the common lookup never
// touches the 128-byte row. Placement is two-choice cuckoo over 4 entries per account of
// capacity (load <= 0.25, below the 0.5 threshold): a lookup issues exactly two 16-byte loads,
// both candidates at once, and never loops. tr_ingest is bound by its texture-address unit
// (TA_BUSY ~70 % in profiles/), which spends a whole wave-instruction on every probe step any
// lane of the wave still needs: linear probing made the 128 lookups of a wave run to the
// longest probe among them (~9 steps each, measured as 29 vector-memory reads per 64 events).
//
// An entry stands for its account's full id and ledger only while kHazardWide is clear (the id's
// high word is 0 and the ledger < 2^16; static, set at insertion). A wide entry matches only after
// comparing the row's id high word, and its readers take the ledger from the row.
//
// Entries are inserted when create_accounts calls finish (accounts never leave the index after
// that) and are immutable except the hazard bits, a conservative summary of the account's dynamic
// state that is only ever set: kHazardClosed when the account may be closed, kHazardHigh when one
// of its balances may have reached 2^126 (hi word >= 2^62). While no hazard bit is set the account
// is open, its ledger fits the entry, and no u128 balance can overflow within a call of < 2^32
// events with amounts < 2^64; otherwise the reader takes the row itself. Writers: create_accounts
// (closed and wide accounts), the ordered replay (update_account), balance application
// (bal_reduce_tiles, bal_bucket_apply, u128 atomics), debug balance setters.
struct alignas(16) AccEntry {
    uint64_t id_lo;
    uint32_t ref;   // row + 1 (0: empty)
    uint32_t meta;  // flags (bits 0-7; `closed` is tracked by hazard) | hazard (8-15) | ledger (16-31)
};
static_assert(sizeof(AccEntry) == 16, "AccEntry is 16 bytes");

enum : uint16_t { kHazardClosed = 1, kHazardHigh = 2, kHazardWide = 4 };
constexpr uint64_t kHazardHiLimit = 1ull << 62;

__host__ __device__ inline uint32_t acc_meta(uint16_t flags, uint16_t hazard, uint32_t ledger) {
    return (flags & 0xFFu) | (uint32_t(hazard & 0xFFu) << 8) | (ledger << 16);
}
__host__ __device__ inline uint16_t meta_flags(uint32_t m) { return uint16_t(m & 0xFFu); }
__host__ __device__ inline uint16_t meta_hazard(uint32_t m) { return uint16_t((m >> 8) & 0xFFu); }
__host__ __device__ inline uint32_t meta_ledger(uint32_t m) { return m >> 16; }

__host__ __device__ inline uint64_t acc_entry_h1(const tb_uint128_t& id) {
    return mix64(id.lo ^ mix64(id.hi ^ 0xD6E8FEB86659FD93ull));
}
__host__ __device__ inline uint64_t acc_entry_h2(const tb_uint128_t& id) {
    return mix64(id.hi ^ mix64(id.lo ^ 0x9FB21C651E98DF25ull) ^ 0xA24BAED4963EE407ull);
}

struct AccIndex {
    AccEntry* entries;
    uint64_t mask;
};

// Does entry image `v` hold `id`? `rows` resolves the high word of wide entries.
__device__ inline bool acc_entry_match(const uint4& v, const tb_account_t* rows,
                                       const tb_uint128_t& id) {
    return v.z != 0 && ((uint64_t(v.y) << 32) | v.x) == id.lo &&
           ((meta_hazard(v.w) & kHazardWide) ? rows[v.z - 1].id.hi == id.hi : id.hi == 0);
}

// Two 16-byte loads, issued together; returns the entry index (its contents in *out) or kNone.
__device__ inline uint64_t acc_index_find(const AccIndex& x, const tb_account_t* rows,
                                          const tb_uint128_t& id, AccEntry* out) {
    if (u128_is_zero(id)) return kNone;
    const uint64_t s1 = acc_entry_h1(id) & x.mask, s2 = acc_entry_h2(id) & x.mask;
    const uint4 v1 = *reinterpret_cast<const uint4*>(&x.entries[s1]);
    const uint4 v2 = *reinterpret_cast<const uint4*>(&x.entries[s2]);
    uint64_t s = kNone;
    uint4 v = v1;
    if (acc_entry_match(v1, rows, id)) {
        s = s1;
    } else if (acc_entry_match(v2, rows, id)) {
        s = s2;
        v = v2;
    }
    if (s != kNone) {
        out->id_lo = id.lo;
        out->ref = v.z;
        out->meta = v.w;
    }
    return s;
}

// Cuckoo insertion of row `row` (its id absent from the index). Only the `ref` words move, by
// atomic exchange, so concurrent insertions never lose an account (each holds exactly one in
// hand); a displaced account continues at its other candidate. Every entry written is appended
// to `dirty` (capacity `dirty_cap`; *overflow is set past it) and the caller rewrites the rest of
// each dirty entry from the row it names (acc_index_repair). Returns false after
// kCuckooMaxKicks displacements (the table is too full).
constexpr int kCuckooMaxKicks = 512;

__device__ inline bool acc_index_insert(const AccIndex& x, const tb_account_t* rows, uint32_t row,
                                        uint32_t* dirty, unsigned int* dirty_count,
                                        uint32_t dirty_cap, unsigned int* overflow) {
    uint32_t r = row;
    uint64_t pos = acc_entry_h1(rows[r].id) & x.mask;
    for (int kick = 0; kick < kCuckooMaxKicks; kick++) {
        const uint32_t old = atomicExch(&x.entries[pos].ref, r + 1);
        const unsigned int d = atomicAdd(dirty_count, 1u);
        if (d < dirty_cap) dirty[d] = uint32_t(pos);
        else atomicOr(overflow, 1u);
        if (old == 0) return true;
        r = old - 1;
        const tb_uint128_t id = rows[r].id;
        const uint64_t h1 = acc_entry_h1(id) & x.mask, h2 = acc_entry_h2(id) & x.mask;
        pos = pos == h1 ? h2 : h1;
    }
    return false;
}

__device__ inline void acc_hazard_set(const AccIndex& x, const uint32_t* entry_of, uint64_t row,
                                      uint16_t bits) {
    const uint32_t s = entry_of[row];
    if (s == 0xFFFFFFFFu) return;  // not indexed yet (an account of the running create_accounts)
    unsigned int* w = &x.entries[s].meta;
    if (((*w >> 8) & bits) != bits) atomicOr(w, (unsigned int)bits << 8);
}

// The hazard bits an account row warrants.
__device__ inline uint16_t acc_hazard_of(const tb_account_t& a) {
    uint16_t h = (a.flags & TB_ACCOUNT_CLOSED) ? kHazardClosed : 0;
    if (a.debits_pending.hi >= kHazardHiLimit || a.debits_posted.hi >= kHazardHiLimit ||
        a.credits_pending.hi >= kHazardHiLimit || a.credits_posted.hi >= kHazardHiLimit)
        h |= kHazardHigh;
    if (a.id.hi != 0 || a.ledger >= (1u << 16)) h |= kHazardWide;
    return h;
}

}  // namespace tbg
