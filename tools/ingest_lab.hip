// Lab: where does create_transfers ingest time go on MI355X? Variants of the ingest memory
// pattern over the bench workload (10M 128-byte events, sequential ids, 10k accounts, a 2^28-slot
// transfer id table holding 60M earlier ids). Not product code: a measurement tool.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include "../tigerbeetle_amd/csrc/device_common.hpp"

using namespace tbg;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

struct Lab {
    const tb_transfer_t* ev;
    tb_transfer_t* rows;
    tb_create_result_t* res;
    unsigned long long* tslots;
    uint64_t tmask;
    const unsigned long long* aslots;
    uint64_t amask;
    const tb_account_t* acc;
    uint32_t* rec_slot;
    uint32_t* rec_dr;
    uint32_t* rec_cr;
    uint64_t* rec_amt;
    uint8_t* rec_info;
    uint32_t n;
    uint64_t row_base;
    uint64_t ts0;
};

__device__ inline uint32_t acc_lookup(const Lab& L, const tb_uint128_t& id, uint64_t* hi_out) {
    uint64_t s = hash_id(id) & L.amask;
    const uint64_t tag = id_tag(id);
    for (int i = 0; i < 64; i++) {
        uint64_t w = L.aslots[s];
        if (w == kEmpty) return ~0u;
        if (slot_tag_is(w, tag)) {
            uint32_t r = uint32_t((w & kRefMask) - 1);
            const tb_account_t* a = &L.acc[r];
            if (u128_eq(a->id, id)) {
                *hi_out = a->debits_posted.hi ^ *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(a) + 112);
                return r;
            }
        }
        s = (s + 1) & L.amask;
    }
    return ~0u;
}

__device__ inline uint64_t claim(const Lab& L, const tb_uint128_t& id, uint64_t ref, bool blind) {
    uint64_t s = hash_id(id) & L.tmask;
    const uint64_t tref = ref | id_tag(id);
    uint64_t w = blind ? kEmpty : L.tslots[s];
    for (int i = 0; i < 4096; i++) {
        if (w == kEmpty) {
            w = atomicCAS(&L.tslots[s], 0ull, (unsigned long long)tref);
            if (w == kEmpty) return s;
        }
        s = (s + 1) & L.tmask;
        w = L.tslots[s];
    }
    return kNone;
}

__global__ void fill(unsigned long long* slots, uint64_t mask, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    tb_uint128_t id{i + 1, 0};
    uint64_t s = hash_id(id) & mask;
    const uint64_t tref = (i + 1) | id_tag(id);
    for (;;) {
        if (atomicCAS(&slots[s], 0ull, (unsigned long long)tref) == 0) return;
        s = (s + 1) & mask;
    }
}

__global__ void acc_fill(unsigned long long* slots, uint64_t mask, tb_account_t* acc, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    tb_account_t a{};
    a.id.lo = i + 1;
    a.ledger = 2;
    a.code = 1;
    acc[i] = a;
    uint64_t s = hash_id(a.id) & mask;
    const uint64_t tref = (i + 1) | id_tag(a.id);
    for (;;) {
        if (atomicCAS(&slots[s], 0ull, (unsigned long long)tref) == 0) return;
        s = (s + 1) & mask;
    }
}

// mode bits
enum { M_CAS = 1, M_BLIND = 2, M_ACC = 4, M_REC = 8 };

template <int MODE>
__device__ inline void one_event(const Lab& L, uint32_t k) {
    tb_transfer_t t;
    {
        const uint4* src = reinterpret_cast<const uint4*>(&L.ev[k]);
        uint4* dst = reinterpret_cast<uint4*>(&t);
#pragma unroll
        for (int i = 0; i < 8; i++) dst[i] = src[i];
    }
    const uint64_t ts = L.ts0 + k;
    uint64_t slot = 0;
    if (MODE & M_CAS) slot = claim(L, t.id, L.row_base + k + 1, (MODE & M_BLIND) != 0);
    uint32_t dr = 0, cr = 0;
    uint64_t h1 = 0, h2 = 0;
    if (MODE & M_ACC) {
        dr = acc_lookup(L, t.debit_account_id, &h1);
        cr = acc_lookup(L, t.credit_account_id, &h2);
    }
    {
        tb_transfer_t o = t;
        o.timestamp = ts;
        const uint4* src = reinterpret_cast<const uint4*>(&o);
        uint4* dst = reinterpret_cast<uint4*>(&L.rows[L.row_base + k]);
#pragma unroll
        for (int i = 0; i < 8; i++) dst[i] = src[i];
    }
    tb_create_result_t r;
    r.timestamp = ts;
    r.status = (h1 ^ h2) == 12345 ? 1 : 0xFFFFFFFFu;
    r.reserved = 0;
    L.res[k] = r;
    if (MODE & M_REC) {
        L.rec_slot[k] = uint32_t(slot);
        L.rec_dr[k] = dr;
        L.rec_cr[k] = cr;
        L.rec_amt[k] = t.amount.lo;
        L.rec_info[k] = 3;
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) k_lpr(Lab L) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < L.n; k += gridDim.x * blockDim.x)
        one_event<MODE>(L, k);
}

template <int MODE>
__global__ void __launch_bounds__(256) k_lpr_flat(Lab L) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < L.n) one_event<MODE>(L, k);
}

// Wave-cooperative copy: 64 events (8 KB) per wave, fully coalesced 16-B lanes; the lane holding
// chunk 7 of an event patches the timestamp.
__global__ void __launch_bounds__(256) k_coal_copy(Lab L) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t w0 = wave * 64; w0 < L.n; w0 += nwaves * 64) {
        const uint4* src = reinterpret_cast<const uint4*>(&L.ev[w0]);
        uint4* dst = reinterpret_cast<uint4*>(&L.rows[L.row_base + w0]);
        uint4 q[8];
#pragma unroll
        for (int i = 0; i < 8; i++) q[i] = src[i * 64 + lane];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t chunk = i * 64 + lane;
            if ((chunk & 7) == 7) {
                const uint64_t ts = L.ts0 + w0 + (chunk >> 3);
                q[i].z = uint32_t(ts);
                q[i].w = uint32_t(ts >> 32);
            }
            dst[i * 64 + lane] = q[i];
        }
        tb_create_result_t r;
        r.timestamp = L.ts0 + w0 + lane;
        r.status = 0xFFFFFFFFu;
        r.reserved = 0;
        L.res[w0 + lane] = r;
    }
}

// LDS-staged: coalesced load of 256 events into LDS, coalesced row store, then lane-per-event
// logic reading fields from LDS.
template <int MODE>
__global__ void __launch_bounds__(256) k_lds(Lab L) {
    __shared__ uint4 tile[256 * 8];
    for (uint32_t base = blockIdx.x * 256; base < L.n; base += gridDim.x * 256) {
        const uint4* src = reinterpret_cast<const uint4*>(&L.ev[base]);
        uint4* dst = reinterpret_cast<uint4*>(&L.rows[L.row_base + base]);
        uint4 q[8];
#pragma unroll
        for (int i = 0; i < 8; i++) q[i] = src[i * 256 + threadIdx.x];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            tile[i * 256 + threadIdx.x] = q[i];
            const uint32_t chunk = i * 256 + threadIdx.x;
            if ((chunk & 7) == 7) {
                const uint64_t ts = L.ts0 + base + (chunk >> 3);
                q[i].z = uint32_t(ts);
                q[i].w = uint32_t(ts >> 32);
            }
            dst[i * 256 + threadIdx.x] = q[i];
        }
        __syncthreads();
        const uint32_t k = base + threadIdx.x;
        const tb_transfer_t& t = *reinterpret_cast<const tb_transfer_t*>(&tile[threadIdx.x * 8]);
        const uint64_t ts = L.ts0 + k;
        uint64_t slot = 0;
        if (MODE & M_CAS) slot = claim(L, t.id, L.row_base + k + 1, (MODE & M_BLIND) != 0);
        uint32_t dr = 0, cr = 0;
        uint64_t h1 = 0, h2 = 0;
        if (MODE & M_ACC) {
            dr = acc_lookup(L, t.debit_account_id, &h1);
            cr = acc_lookup(L, t.credit_account_id, &h2);
        }
        tb_create_result_t r;
        r.timestamp = ts;
        r.status = (h1 ^ h2) == 12345 ? 1 : 0xFFFFFFFFu;
        r.reserved = 0;
        L.res[k] = r;
        if (MODE & M_REC) {
            L.rec_slot[k] = uint32_t(slot);
            L.rec_dr[k] = dr;
            L.rec_cr[k] = cr;
            L.rec_amt[k] = t.amount.lo;
            L.rec_info[k] = 3;
        }
        __syncthreads();
    }
}


// ---- variant structures -------------------------------------------------------------------
__host__ __device__ inline uint64_t home16(const tb_uint128_t& id) {
    const uint64_t g = mix64((id.lo >> 4) ^ mix64(id.hi + 0x9E3779B97F4A7C15ull));
    return (g << 4) | ((id.lo ^ (g >> 60)) & 15);
}
__global__ void fill16(unsigned long long* slots, uint64_t mask, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    tb_uint128_t id{i + 1, 0};
    uint64_t s = home16(id) & mask;
    const uint64_t tref = (i + 1) | id_tag(id);
    for (;;) {
        if (atomicCAS(&slots[s], 0ull, (unsigned long long)tref) == 0) return;
        s = (s + 16) & mask;
    }
}
__device__ inline uint64_t claim16(const Lab& L, const tb_uint128_t& id, uint64_t ref) {
    uint64_t s = home16(id) & L.tmask;
    const uint64_t tref = ref | id_tag(id);
    for (int i = 0; i < 4096; i++) {
        uint64_t w = atomicCAS(&L.tslots[s], 0ull, (unsigned long long)tref);
        if (w == kEmpty) return s;
        s = (s + 16) & L.tmask;
    }
    return kNone;
}
struct alignas(16) AccEntry {
    tb_uint128_t id;
    uint32_t row, ledger;
    uint16_t flags, hazard;
    uint32_t pad;
};
__global__ void acc32_fill(AccEntry* e, uint64_t mask, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    tb_uint128_t id{i + 1, 0};
    uint64_t s = mix64(id.lo ^ mix64(id.hi)) & mask;
    for (;;) {
        unsigned long long* w = reinterpret_cast<unsigned long long*>(&e[s].id.lo);
        if (atomicCAS(w, 0ull, id.lo) == 0) {
            e[s].id.hi = id.hi; e[s].row = i; e[s].ledger = 2; e[s].flags = 0; e[s].hazard = 0;
            return;
        }
        s = (s + 1) & mask;
    }
}
__device__ inline uint32_t acc32_lookup(const AccEntry* E, uint64_t mask, const tb_uint128_t& id,
                                        uint32_t* ledger) {
    uint64_t s = mix64(id.lo ^ mix64(id.hi)) & mask;
    for (int i = 0; i < 64; i++) {
        const uint4* p = reinterpret_cast<const uint4*>(&E[s]);
        uint4 a = p[0], b = p[1];
        const uint64_t lo = (uint64_t(a.y) << 32) | a.x, hi = (uint64_t(a.w) << 32) | a.z;
        if (lo == id.lo && hi == id.hi) { *ledger = b.y; return b.x; }
        if ((lo | hi) == 0) return ~0u;
        s = (s + 1) & mask;
    }
    return ~0u;
}
__device__ const AccEntry* g_acc32;
__device__ uint64_t g_acc32_mask;

// Wave-cooperative: 64 events per wave-iteration, coalesced load + row store, per-wave LDS
// transpose (XOR-swizzled 16-B parts), then lane-per-event table work.
template <int MODE, bool PREFETCH>
__global__ void __launch_bounds__(256) k_wc(Lab L, const AccEntry* E, uint64_t emask) {
    __shared__ uint4 lds[4][512];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint4* my = lds[wv];
    const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    uint4 q[8];
    uint32_t base = gw * 64;
    if (base < L.n) {
        const uint4* src = reinterpret_cast<const uint4*>(&L.ev[base]);
#pragma unroll
        for (int i = 0; i < 8; i++) q[i] = src[i * 64 + lane];
    }
    for (; base < L.n; base += nw * 64) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t e = i * 8 + (lane >> 3), p = lane & 7;
            my[e * 8 + (p ^ (e & 7))] = q[i];
        }
        uint4* dst = reinterpret_cast<uint4*>(&L.rows[L.row_base + base]);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if ((lane & 7) == 7) {
                const uint64_t ts = L.ts0 + base + i * 8 + (lane >> 3);
                q[i].z = uint32_t(ts);
                q[i].w = uint32_t(ts >> 32);
            }
            dst[i * 64 + lane] = q[i];
        }
        const uint32_t next = base + nw * 64;
        if (PREFETCH && next < L.n) {
            const uint4* src = reinterpret_cast<const uint4*>(&L.ev[next]);
#pragma unroll
            for (int i = 0; i < 8; i++) q[i] = src[i * 64 + lane];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t k = base + lane;
        const uint32_t e = lane;
        auto part = [&](int p) { return my[e * 8 + (p ^ (e & 7))]; };
        const uint4 p0 = part(0), p1 = part(1), p2 = part(2), p3 = part(3);
        tb_uint128_t id{(uint64_t(p0.y) << 32) | p0.x, (uint64_t(p0.w) << 32) | p0.z};
        tb_uint128_t dra{(uint64_t(p1.y) << 32) | p1.x, (uint64_t(p1.w) << 32) | p1.z};
        tb_uint128_t cra{(uint64_t(p2.y) << 32) | p2.x, (uint64_t(p2.w) << 32) | p2.z};
        const uint64_t amount = (uint64_t(p3.y) << 32) | p3.x;
        const uint64_t ts = L.ts0 + k;
        uint64_t slot = 0;
        if (MODE & M_CAS) slot = claim16(L, id, L.row_base + k + 1);
        uint32_t dr = 0, cr = 0, l1 = 0, l2 = 0;
        if (MODE & M_ACC) {
            dr = acc32_lookup(E, emask, dra, &l1);
            cr = acc32_lookup(E, emask, cra, &l2);
        }
        tb_create_result_t r;
        r.timestamp = ts;
        r.status = (l1 ^ l2) == 12345 ? 1 : 0xFFFFFFFFu;
        r.reserved = 0;
        L.res[k] = r;
        if (MODE & M_REC) {
            L.rec_slot[k] = uint32_t(slot);
            L.rec_dr[k] = dr;
            L.rec_cr[k] = cr;
            L.rec_amt[k] = amount;
            L.rec_info[k] = 3;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (!PREFETCH && next < L.n) {
            const uint4* src = reinterpret_cast<const uint4*>(&L.ev[next]);
#pragma unroll
            for (int i = 0; i < 8; i++) q[i] = src[i * 64 + lane];
        }
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) k_lpr16(Lab L, const AccEntry* E, uint64_t emask) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < L.n; k += gridDim.x * blockDim.x) {
        tb_transfer_t t;
        {
            const uint4* src = reinterpret_cast<const uint4*>(&L.ev[k]);
            uint4* dst = reinterpret_cast<uint4*>(&t);
#pragma unroll
            for (int i = 0; i < 8; i++) dst[i] = src[i];
        }
        const uint64_t ts = L.ts0 + k;
        uint64_t slot = 0;
        if (MODE & M_CAS) slot = claim16(L, t.id, L.row_base + k + 1);
        uint32_t dr = 0, cr = 0, l1 = 0, l2 = 0;
        if (MODE & M_ACC) {
            dr = acc32_lookup(E, emask, t.debit_account_id, &l1);
            cr = acc32_lookup(E, emask, t.credit_account_id, &l2);
        }
        {
            tb_transfer_t o = t;
            o.timestamp = ts;
            const uint4* src = reinterpret_cast<const uint4*>(&o);
            uint4* dst = reinterpret_cast<uint4*>(&L.rows[L.row_base + k]);
#pragma unroll
            for (int i = 0; i < 8; i++) dst[i] = src[i];
        }
        tb_create_result_t r;
        r.timestamp = ts;
        r.status = (l1 ^ l2) == 12345 ? 1 : 0xFFFFFFFFu;
        r.reserved = 0;
        L.res[k] = r;
        if (MODE & M_REC) {
            L.rec_slot[k] = uint32_t(slot);
            L.rec_dr[k] = dr;
            L.rec_cr[k] = cr;
            L.rec_amt[k] = t.amount.lo;
            L.rec_info[k] = 3;
        }
    }
}

int main() {
    const uint32_t N = 10000000, A = 10000;
    const uint64_t TSLOTS = 1ull << 28, ASLOTS = 1ull << 15, PREFILL = 60000000;
    std::vector<tb_transfer_t> h(N);
    uint64_t x = 42;
    for (uint32_t k = 0; k < N; k++) {
        tb_transfer_t t{};
        t.id.lo = PREFILL + k + 1;
        x = mix64(x + k);
        uint32_t d = x % A, c = (x >> 20) % A;
        if (c == d) c = (c + 1) % A;
        t.debit_account_id.lo = d + 1;
        t.credit_account_id.lo = c + 1;
        t.amount.lo = (x >> 40) % 20000 + 1;
        t.ledger = 2;
        t.code = 1;
        h[k] = t;
    }
    Lab L{};
    tb_transfer_t *ev, *rows;
    CK(hipMalloc(&ev, N * 128ull));
    CK(hipMemcpy(ev, h.data(), N * 128ull, hipMemcpyHostToDevice));
    CK(hipMalloc(&rows, 80000000ull * 128));
    tb_create_result_t* res;
    CK(hipMalloc(&res, N * 16ull));
    unsigned long long *ts, *as;
    CK(hipMalloc(&ts, TSLOTS * 8));
    CK(hipMalloc(&as, ASLOTS * 8));
    tb_account_t* acc;
    CK(hipMalloc(&acc, A * 128ull));
    CK(hipMemset(as, 0, ASLOTS * 8));
    acc_fill<<<(A + 255) / 256, 256>>>(as, ASLOTS - 1, acc, A);
    uint32_t *rs, *rd, *rc;
    uint64_t* ra;
    uint8_t* ri;
    CK(hipMalloc(&rs, N * 4ull));
    CK(hipMalloc(&rd, N * 4ull));
    CK(hipMalloc(&rc, N * 4ull));
    CK(hipMalloc(&ra, N * 8ull));
    CK(hipMalloc(&ri, N * 1ull));
    L.ev = ev; L.rows = rows; L.res = res; L.tslots = ts; L.tmask = TSLOTS - 1;
    L.aslots = as; L.amask = ASLOTS - 1; L.acc = acc;
    L.rec_slot = rs; L.rec_dr = rd; L.rec_cr = rc; L.rec_amt = ra; L.rec_info = ri;
    L.n = N; L.row_base = PREFILL; L.ts0 = 1000;

    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto reset = [&]() {
        hipMemset(ts, 0, TSLOTS * 8);
        fill<<<(PREFILL + 255) / 256, 256>>>(ts, TSLOTS - 1, PREFILL);
        hipDeviceSynchronize();
    };
    auto run = [&](const char* name, auto launch, bool needs_reset) {
        std::vector<float> v;
        for (int rep = 0; rep < 4; rep++) {
            if (needs_reset) reset();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            v.push_back(ms);
        }
        std::sort(v.begin(), v.end());
        hipError_t e = hipGetLastError();
        printf("%-34s %.3f ms (min %.3f)  %s\n", name, v[v.size() / 2], v[0],
               e == hipSuccess ? "" : hipGetErrorString(e));
        fflush(stdout);
    };
    const int G = 4096, B = 256, GF = (N + 255) / 256;
    run("copy lane-per-row (grid 4096)", [&] { k_lpr<0><<<G, B>>>(L); }, false);
    run("copy lane-per-row (flat)", [&] { k_lpr_flat<0><<<GF, B>>>(L); }, false);
    run("copy coalesced", [&] { k_coal_copy<<<G, B>>>(L); }, false);
    run("lpr + blind CAS", [&] { k_lpr<M_CAS | M_BLIND><<<G, B>>>(L); }, true);
    run("lpr + load,CAS", [&] { k_lpr<M_CAS><<<G, B>>>(L); }, true);
    run("lpr + blind CAS (flat)", [&] { k_lpr_flat<M_CAS | M_BLIND><<<GF, B>>>(L); }, true);
    run("lpr + acc", [&] { k_lpr<M_ACC><<<G, B>>>(L); }, false);
    run("lpr + acc + rec", [&] { k_lpr<M_ACC | M_REC><<<G, B>>>(L); }, false);
    run("lpr + blindCAS + acc + rec", [&] { k_lpr<M_CAS | M_BLIND | M_ACC | M_REC><<<G, B>>>(L); }, true);
    run("lpr + blindCAS + acc + rec (flat)", [&] { k_lpr_flat<M_CAS | M_BLIND | M_ACC | M_REC><<<GF, B>>>(L); }, true);
    run("lds copy", [&] { k_lds<0><<<G, B>>>(L); }, false);
    run("lds + blind CAS", [&] { k_lds<M_CAS | M_BLIND><<<G, B>>>(L); }, true);
    run("lds + acc + rec", [&] { k_lds<M_ACC | M_REC><<<G, B>>>(L); }, false);
    run("lds + blindCAS + acc + rec", [&] { k_lds<M_CAS | M_BLIND | M_ACC | M_REC><<<G, B>>>(L); }, true);
    run("lds + blindCAS + acc + rec (flat)", [&] { k_lds<M_CAS | M_BLIND | M_ACC | M_REC><<<GF, B>>>(L); }, true);
    AccEntry* E;
    const uint64_t EN = 1ull << 15;
    CK(hipMalloc(&E, EN * 32));
    CK(hipMemset(E, 0, EN * 32));
    acc32_fill<<<(A + 255) / 256, 256>>>(E, EN - 1, A);
    auto reset16 = [&]() {
        hipMemset(ts, 0, TSLOTS * 8);
        fill16<<<(PREFILL + 255) / 256, 256>>>(ts, TSLOTS - 1, PREFILL);
        hipDeviceSynchronize();
    };
    auto run16 = [&](const char* name, auto launch, bool needs_reset) {
        std::vector<float> v;
        for (int rep = 0; rep < 4; rep++) {
            if (needs_reset) reset16();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            v.push_back(ms);
        }
        std::sort(v.begin(), v.end());
        hipError_t e = hipGetLastError();
        printf("%-34s %.3f ms (min %.3f)  %s\n", name, v[v.size() / 2], v[0],
               e == hipSuccess ? "" : hipGetErrorString(e));
        fflush(stdout);
    };
    run16("lpr + CAS16", [&] { k_lpr16<M_CAS><<<G, B>>>(L, E, EN - 1); }, true);
    run16("lpr + acc32", [&] { k_lpr16<M_ACC><<<G, B>>>(L, E, EN - 1); }, false);
    run16("lpr + CAS16 + acc32 + rec", [&] { k_lpr16<M_CAS | M_ACC | M_REC><<<G, B>>>(L, E, EN - 1); }, true);
    run16("wc copy", [&] { k_wc<0, false><<<G, B>>>(L, E, EN - 1); }, false);
    run16("wc copy prefetch", [&] { k_wc<0, true><<<G, B>>>(L, E, EN - 1); }, false);
    run16("wc + CAS16", [&] { k_wc<M_CAS, false><<<G, B>>>(L, E, EN - 1); }, true);
    run16("wc + acc32 + rec", [&] { k_wc<M_ACC | M_REC, false><<<G, B>>>(L, E, EN - 1); }, false);
    run16("wc + all", [&] { k_wc<M_CAS | M_ACC | M_REC, false><<<G, B>>>(L, E, EN - 1); }, true);
    run16("wc + all prefetch", [&] { k_wc<M_CAS | M_ACC | M_REC, true><<<G, B>>>(L, E, EN - 1); }, true);
    run16("wc + all prefetch grid 2048", [&] { k_wc<M_CAS | M_ACC | M_REC, true><<<2048, B>>>(L, E, EN - 1); }, true);
    run16("wc + all prefetch grid 1280", [&] { k_wc<M_CAS | M_ACC | M_REC, true><<<1280, B>>>(L, E, EN - 1); }, true);
    return 0;
}
