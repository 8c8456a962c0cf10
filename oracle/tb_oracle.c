/*
 * tb_oracle.c -- TEST INFRASTRUCTURE: serial CPU restatement of TigerBeetle's commit path.
 *
 * This file is the parity checker for the HIP executor (tigerbeetle_amd/csrc) and the CPU
 * baseline of bench.py. It is never linked into the product library. It restates, event by
 * event and in the reference's exact check order:
 *
 *   execute_create             src/state_machine.zig:3002-3213
 *   transient_error            src/state_machine.zig:3215-3252
 *   create_account(_exists)    src/state_machine.zig:3613-3703
 *   create_transfer(_exists)   src/state_machine.zig:3719-4051
 *   post_or_void_pending_...   src/state_machine.zig:4053-4382
 *   execute_expire_pending_... src/state_machine.zig:4511-4628 with the scan/finish rules of
 *                              ExpirePendingTransfersType, src/state_machine.zig:4875-5029 and
 *                              src/lsm/scan_lookup.zig:150-175 (buffer_finished before next()).
 *   sum_overflows              src/state_machine.zig:5144-5149
 *
 * Groove semantics (src/lsm/groove.zig:885-951, :1770-1949; src/lsm/cache_map.zig:331-385;
 * src/lsm/tree.zig:178-226) are modelled with hash maps plus a scope undo log:
 *   - inserts/updates are visible to later events of the same batch;
 *   - scope_close(discard) reverts objects, statuses and the objects trees' key_range;
 *   - orphaned transfer ids (transient failures) are inserted outside any scope and never revert;
 *   - pulse_next_timestamp is state-machine state, not groove state: it is never reverted.
 *
 * Parity pin: tests/test_oracle_tables.py replays the reference's table tests
 * (src/state_machine_tests.zig) against this file.
 */
#include "tb_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

static inline u128 U(tb_uint128_t x) { return ((u128)x.hi << 64) | x.lo; }
static inline tb_uint128_t W(u128 x) {
    tb_uint128_t r;
    r.lo = (uint64_t)x;
    r.hi = (uint64_t)(x >> 64);
    return r;
}
static const u128 U128_MAX = ~(u128)0;

static void* xrealloc(void* p, size_t n) {
    void* q = realloc(p, n);
    if (!q && n) {
        fprintf(stderr, "tb_oracle: out of memory\n");
        abort();
    }
    return q;
}

/* ---- u128 -> u64 hash map: linear probing, backward-shift deletion --------------------------*/

typedef struct {
    u128* keys;
    uint64_t* vals;
    uint8_t* used;
    uint64_t cap; /* power of two */
    uint64_t count;
} map_t;

static inline uint64_t mix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h;
}
static inline uint64_t hash128(u128 k) {
    return mix64((uint64_t)k ^ mix64((uint64_t)(k >> 64) + 0x9E3779B97F4A7C15ull));
}

static void map_init(map_t* m, uint64_t cap) {
    m->cap = cap;
    m->count = 0;
    m->keys = (u128*)xrealloc(NULL, cap * sizeof(u128));
    m->vals = (uint64_t*)xrealloc(NULL, cap * sizeof(uint64_t));
    m->used = (uint8_t*)calloc(cap, 1);
}
static void map_free(map_t* m) {
    free(m->keys);
    free(m->vals);
    free(m->used);
}
static int map_get(const map_t* m, u128 key, uint64_t* val) {
    uint64_t mask = m->cap - 1, i = hash128(key) & mask;
    while (m->used[i]) {
        if (m->keys[i] == key) {
            if (val) *val = m->vals[i];
            return 1;
        }
        i = (i + 1) & mask;
    }
    return 0;
}
static void map_put(map_t* m, u128 key, uint64_t val);
static void map_grow(map_t* m) {
    map_t n;
    map_init(&n, m->cap * 2);
    for (uint64_t i = 0; i < m->cap; i++)
        if (m->used[i]) map_put(&n, m->keys[i], m->vals[i]);
    map_free(m);
    *m = n;
}
static void map_put(map_t* m, u128 key, uint64_t val) {
    if ((m->count + 1) * 2 > m->cap) map_grow(m);
    uint64_t mask = m->cap - 1, i = hash128(key) & mask;
    while (m->used[i]) {
        if (m->keys[i] == key) {
            m->vals[i] = val;
            return;
        }
        i = (i + 1) & mask;
    }
    m->used[i] = 1;
    m->keys[i] = key;
    m->vals[i] = val;
    m->count++;
}
static void map_del(map_t* m, u128 key) {
    uint64_t mask = m->cap - 1, i = hash128(key) & mask;
    while (m->used[i] && m->keys[i] != key) i = (i + 1) & mask;
    if (!m->used[i]) return;
    m->used[i] = 0;
    m->count--;
    /* Backward-shift: re-seat the rest of the cluster. */
    uint64_t j = (i + 1) & mask;
    while (m->used[j]) {
        u128 k = m->keys[j];
        uint64_t v = m->vals[j];
        m->used[j] = 0;
        m->count--;
        map_put(m, k, v);
        j = (j + 1) & mask;
    }
}

/* ---- state ----------------------------------------------------------------------------------*/

#define ORPHAN UINT64_MAX

enum { UNDO_ACCOUNT = 1, UNDO_STATUS = 2 };
typedef struct {
    uint32_t kind;
    uint64_t index;
    tb_account_t account; /* UNDO_ACCOUNT: the row before the update */
    uint8_t status;       /* UNDO_STATUS: the TransferPending status before the update */
} undo_t;

typedef struct {
    int has;
    uint64_t key_max; /* tree.key_range.key_max of the objects tree (timestamps) */
} key_range_t;

struct tbo_ctx {
    tb_account_t* accounts;
    uint64_t n_accounts, cap_accounts;
    tb_transfer_t* transfers;
    uint8_t* pending_status; /* TransferPending.status, keyed by the transfer (= its timestamp) */
    uint64_t n_transfers, cap_transfers;

    map_t account_by_id, account_by_ts;
    map_t transfer_by_id, transfer_by_ts; /* transfer_by_id value ORPHAN = orphaned id */
    key_range_t accounts_range, transfers_range;

    uint64_t* expiry; /* transfers with flags.pending and timeout > 0 (expires_at index) */
    uint64_t n_expiry, cap_expiry;

    uint64_t pulse_next_timestamp;
    uint32_t pulse_batch_max;
    uint64_t commit_timestamp;

    /* Sharded pulse_next_timestamp (tbo_pnt_sharded): every update is logged with its event's
     * timestamp -- `min` updates applied, reset-if-equal ones only logged (the reset compares
     * against the value across all shards, which the caller resolves). */
    int pnt_sharded;
    uint64_t* pnt_ts;
    uint64_t* pnt_op;
    uint64_t n_pnt, cap_pnt;
    uint64_t pnt_start; /* pulse_next_timestamp before the logged updates */

    /* The account_events groove (state_machine.zig:104-220), in insertion order. */
    tb_account_event_t* events;
    uint64_t n_events, cap_events;

    /* One active scope at a time (tree.zig:178-197). */
    int scope_active;
    uint64_t scope_n_accounts, scope_n_transfers, scope_n_expiry, scope_n_events;
    key_range_t scope_accounts_range, scope_transfers_range;
    undo_t* undo;
    uint64_t n_undo, cap_undo;
};

/* Test instrumentation for sharded calls (not a reference mechanism): the pulse_next_timestamp
 * updates of post_or_void_pending_transfer (:4227-4229) and create_transfer (:3975-3982). */
#define TBO_PNT_RESET (1ull << 63)
static void pnt_log(tbo_ctx* c, uint64_t ts, uint64_t op) {
    if (c->n_pnt == 0) c->pnt_start = c->pulse_next_timestamp;
    if (c->n_pnt == c->cap_pnt) {
        c->cap_pnt = c->cap_pnt ? 2 * c->cap_pnt : 1024;
        c->pnt_ts = (uint64_t*)xrealloc(c->pnt_ts, c->cap_pnt * sizeof(uint64_t));
        c->pnt_op = (uint64_t*)xrealloc(c->pnt_op, c->cap_pnt * sizeof(uint64_t));
    }
    c->pnt_ts[c->n_pnt] = ts;
    c->pnt_op[c->n_pnt] = op;
    c->n_pnt++;
}

void tbo_pnt_sharded(tbo_ctx* c, int on) { c->pnt_sharded = on; }

uint64_t tbo_pnt_ops(tbo_ctx* c, uint64_t* ts, uint64_t* ops, uint64_t* start) {
    const uint64_t n = c->n_pnt;
    if (start) *start = n ? c->pnt_start : c->pulse_next_timestamp;
    for (uint64_t i = 0; i < n; i++) {
        if (ts) ts[i] = c->pnt_ts[i];
        if (ops) ops[i] = c->pnt_op[i];
    }
    if (ts || ops) c->n_pnt = 0;
    return n;
}

void tbo_set_pulse_next_timestamp(tbo_ctx* c, uint64_t v) { c->pulse_next_timestamp = v; }

tbo_ctx* tbo_open(uint32_t pulse_batch_max, uint64_t pulse_next_timestamp_init) {
    tbo_ctx* c = (tbo_ctx*)calloc(1, sizeof(tbo_ctx));
    map_init(&c->account_by_id, 1024);
    map_init(&c->account_by_ts, 1024);
    map_init(&c->transfer_by_id, 1024);
    map_init(&c->transfer_by_ts, 1024);
    c->pulse_batch_max = pulse_batch_max;
    c->pulse_next_timestamp = pulse_next_timestamp_init;
    return c;
}

void tbo_close(tbo_ctx* c) {
    if (!c) return;
    free(c->accounts);
    free(c->transfers);
    free(c->pending_status);
    free(c->expiry);
    free(c->undo);
    free(c->events);
    free(c->pnt_ts);
    free(c->pnt_op);
    map_free(&c->account_by_id);
    map_free(&c->account_by_ts);
    map_free(&c->transfer_by_id);
    map_free(&c->transfer_by_ts);
    free(c);
}

static void undo_push(tbo_ctx* c, undo_t* u) {
    if (!c->scope_active) return;
    if (c->n_undo == c->cap_undo) {
        c->cap_undo = c->cap_undo ? c->cap_undo * 2 : 256;
        c->undo = (undo_t*)xrealloc(c->undo, c->cap_undo * sizeof(undo_t));
    }
    c->undo[c->n_undo++] = *u;
}

static void scope_open(tbo_ctx* c) {
    c->scope_active = 1;
    c->scope_n_accounts = c->n_accounts;
    c->scope_n_transfers = c->n_transfers;
    c->scope_n_expiry = c->n_expiry;
    c->scope_n_events = c->n_events;
    c->scope_accounts_range = c->accounts_range;
    c->scope_transfers_range = c->transfers_range;
    c->n_undo = 0;
}

static void scope_close(tbo_ctx* c, int discard) {
    if (discard) {
        /* Reverse order, like cache_map.zig:361-385. */
        for (uint64_t k = c->n_undo; k-- > 0;) {
            undo_t* u = &c->undo[k];
            if (u->kind == UNDO_ACCOUNT) {
                c->accounts[u->index] = u->account;
            } else {
                c->pending_status[u->index] = u->status;
            }
        }
        for (uint64_t i = c->scope_n_accounts; i < c->n_accounts; i++) {
            map_del(&c->account_by_id, U(c->accounts[i].id));
            map_del(&c->account_by_ts, c->accounts[i].timestamp);
        }
        for (uint64_t i = c->scope_n_transfers; i < c->n_transfers; i++) {
            map_del(&c->transfer_by_id, U(c->transfers[i].id));
            map_del(&c->transfer_by_ts, c->transfers[i].timestamp);
        }
        c->n_accounts = c->scope_n_accounts;
        c->n_transfers = c->scope_n_transfers;
        c->n_expiry = c->scope_n_expiry;
        c->n_events = c->scope_n_events; /* account_events inserted in the scope */
        c->accounts_range = c->scope_accounts_range;
        c->transfers_range = c->scope_transfers_range;
    }
    c->scope_active = 0;
    c->n_undo = 0;
}

static tb_account_t* get_account(tbo_ctx* c, u128 id) {
    uint64_t v;
    if (!map_get(&c->account_by_id, id, &v)) return NULL;
    return &c->accounts[v];
}

/* groove.get for transfers: 0 = not_found, 1 = found_object, 2 = found_orphaned */
static int get_transfer(tbo_ctx* c, u128 id, uint64_t* index) {
    uint64_t v;
    if (!map_get(&c->transfer_by_id, id, &v)) return 0;
    if (v == ORPHAN) return 2;
    *index = v;
    return 1;
}

static void key_range_update(key_range_t* r, uint64_t key) {
    if (!r->has || key > r->key_max) r->key_max = key;
    r->has = 1;
}

static void insert_account(tbo_ctx* c, const tb_account_t* a) {
    if (c->n_accounts == c->cap_accounts) {
        c->cap_accounts = c->cap_accounts ? c->cap_accounts * 2 : 1024;
        c->accounts = (tb_account_t*)xrealloc(c->accounts, c->cap_accounts * sizeof(tb_account_t));
    }
    uint64_t i = c->n_accounts++;
    c->accounts[i] = *a;
    map_put(&c->account_by_id, U(a->id), i);
    map_put(&c->account_by_ts, a->timestamp, i);
    key_range_update(&c->accounts_range, a->timestamp);
}

static void update_account(tbo_ctx* c, tb_account_t* row, const tb_account_t* next) {
    uint64_t index = (uint64_t)(row - c->accounts);
    if (c->scope_active && index < c->scope_n_accounts) {
        undo_t u;
        memset(&u, 0, sizeof(u));
        u.kind = UNDO_ACCOUNT;
        u.index = index;
        u.account = *row;
        undo_push(c, &u);
    }
    *row = *next;
}

static uint64_t insert_transfer(tbo_ctx* c, const tb_transfer_t* t, uint8_t status) {
    if (c->n_transfers == c->cap_transfers) {
        c->cap_transfers = c->cap_transfers ? c->cap_transfers * 2 : 1024;
        c->transfers =
            (tb_transfer_t*)xrealloc(c->transfers, c->cap_transfers * sizeof(tb_transfer_t));
        c->pending_status = (uint8_t*)xrealloc(c->pending_status, c->cap_transfers);
    }
    uint64_t i = c->n_transfers++;
    c->transfers[i] = *t;
    c->pending_status[i] = status;
    map_put(&c->transfer_by_id, U(t->id), i);
    map_put(&c->transfer_by_ts, t->timestamp, i);
    key_range_update(&c->transfers_range, t->timestamp);
    if ((t->flags & TB_TRANSFER_PENDING) && t->timeout > 0) {
        if (c->n_expiry == c->cap_expiry) {
            c->cap_expiry = c->cap_expiry ? c->cap_expiry * 2 : 1024;
            c->expiry = (uint64_t*)xrealloc(c->expiry, c->cap_expiry * sizeof(uint64_t));
        }
        c->expiry[c->n_expiry++] = i;
    }
    return i;
}

static void update_pending_status(tbo_ctx* c, uint64_t index, uint8_t status) {
    if (c->scope_active && index < c->scope_n_transfers) {
        undo_t u;
        memset(&u, 0, sizeof(u));
        u.kind = UNDO_STATUS;
        u.index = index;
        u.status = c->pending_status[index];
        undo_push(c, &u);
    }
    c->pending_status[index] = status;
}

static inline int sum_overflows_u128(u128 a, u128 b) { return a + b < a; }

/* account_event (state_machine.zig:4384-4465): the accounts as they stand after the event.
 * `p` is the pending transfer of a post / void / expiry (else NULL); an expiry has no transfer
 * flags and no requested amount. Inserted regardless of Account.flags.history (CDC). */
static void account_event(tbo_ctx* c, uint64_t timestamp_event, const tb_account_t* dr,
                          const tb_account_t* cr, uint16_t transfer_flags, uint8_t pending_status,
                          const tb_transfer_t* p, u128 amount_requested, u128 amount) {
    if (c->n_events == c->cap_events) {
        c->cap_events = c->cap_events ? c->cap_events * 2 : 1024;
        c->events = (tb_account_event_t*)xrealloc(c->events,
                                                  c->cap_events * sizeof(tb_account_event_t));
    }
    tb_account_event_t* e = &c->events[c->n_events++];
    memset(e, 0, sizeof(*e));
    e->timestamp = timestamp_event;
    e->dr_account_id = dr->id;
    e->dr_account_timestamp = dr->timestamp;
    e->dr_debits_pending = dr->debits_pending;
    e->dr_debits_posted = dr->debits_posted;
    e->dr_credits_pending = dr->credits_pending;
    e->dr_credits_posted = dr->credits_posted;
    e->dr_account_flags = dr->flags;
    e->cr_account_id = cr->id;
    e->cr_account_timestamp = cr->timestamp;
    e->cr_debits_pending = cr->debits_pending;
    e->cr_debits_posted = cr->debits_posted;
    e->cr_credits_pending = cr->credits_pending;
    e->cr_credits_posted = cr->credits_posted;
    e->cr_account_flags = cr->flags;
    e->amount_requested = W(amount_requested);
    e->amount = W(amount);
    if (dr->ledger != cr->ledger) abort(); /* asserted by the reference */
    e->ledger = dr->ledger;
    e->transfer_flags = transfer_flags;
    e->transfer_pending_status = pending_status;
    if (p) {
        e->transfer_pending_id = p->id;
        e->transfer_pending_flags = p->flags;
    }
}

/* ---- create_account (state_machine.zig:3613-3703) ------------------------------------------*/

static uint32_t create_account_exists(const tb_account_t* a, const tb_account_t* e,
                                      uint64_t* ts) {
    if (a->flags != e->flags) return TB_CA_EXISTS_WITH_DIFFERENT_FLAGS;
    if (U(a->user_data_128) != U(e->user_data_128))
        return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (a->user_data_64 != e->user_data_64) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (a->user_data_32 != e->user_data_32) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (a->ledger != e->ledger) return TB_CA_EXISTS_WITH_DIFFERENT_LEDGER;
    if (a->code != e->code) return TB_CA_EXISTS_WITH_DIFFERENT_CODE;
    *ts = e->timestamp;
    return TB_CA_EXISTS;
}

static uint32_t create_account(tbo_ctx* c, uint64_t timestamp_event, const tb_account_t* a,
                               uint64_t* ts) {
    if (a->reserved != 0) return TB_CA_RESERVED_FIELD;
    if (a->flags & TB_ACCOUNT_PADDING_MASK) return TB_CA_RESERVED_FLAG;
    u128 id = U(a->id);
    if (id == 0) return TB_CA_ID_MUST_NOT_BE_ZERO;
    if (id == U128_MAX) return TB_CA_ID_MUST_NOT_BE_INT_MAX;

    tb_account_t* e = get_account(c, id);
    if (e) return create_account_exists(a, e, ts);

    if ((a->flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
        (a->flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
        return TB_CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (U(a->debits_pending) != 0) return TB_CA_DEBITS_PENDING_MUST_BE_ZERO;
    if (U(a->debits_posted) != 0) return TB_CA_DEBITS_POSTED_MUST_BE_ZERO;
    if (U(a->credits_pending) != 0) return TB_CA_CREDITS_PENDING_MUST_BE_ZERO;
    if (U(a->credits_posted) != 0) return TB_CA_CREDITS_POSTED_MUST_BE_ZERO;
    if (a->ledger == 0) return TB_CA_LEDGER_MUST_NOT_BE_ZERO;
    if (a->code == 0) return TB_CA_CODE_MUST_NOT_BE_ZERO;

    uint64_t timestamp_actual = timestamp_event;
    if (a->flags & TB_ACCOUNT_IMPORTED) {
        if (c->accounts_range.has && a->timestamp <= c->accounts_range.key_max)
            return TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (map_get(&c->transfer_by_ts, a->timestamp, NULL))
            return TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        timestamp_actual = a->timestamp;
    }

    tb_account_t row;
    memset(&row, 0, sizeof(row));
    row.id = a->id;
    row.user_data_128 = a->user_data_128;
    row.user_data_64 = a->user_data_64;
    row.user_data_32 = a->user_data_32;
    row.ledger = a->ledger;
    row.code = a->code;
    row.flags = a->flags;
    row.timestamp = timestamp_actual;
    insert_account(c, &row);
    c->commit_timestamp = timestamp_actual;
    *ts = timestamp_actual;
    return TB_STATUS_CREATED;
}

/* ---- create_transfer (state_machine.zig:3719-4051) -----------------------------------------*/

static uint32_t post_or_void_pending_transfer_exists(const tb_transfer_t* t,
                                                     const tb_transfer_t* e,
                                                     const tb_transfer_t* p, uint64_t* ts) {
    if (U(t->debit_account_id) != 0 && U(t->debit_account_id) != U(e->debit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (U(t->credit_account_id) != 0 && U(t->credit_account_id) != U(e->credit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t->flags & TB_TRANSFER_VOID_PENDING) {
        if (U(t->amount) == 0) {
            if (U(e->amount) != U(p->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        } else {
            if (U(t->amount) != U(e->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        }
    }
    if (t->flags & TB_TRANSFER_POST_PENDING) {
        if (U(t->amount) == U128_MAX) {
            if (U(e->amount) != U(p->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        } else {
            if (U(t->amount) != U(e->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        }
    }
    if (U(t->user_data_128) == 0) {
        if (U(e->user_data_128) != U(p->user_data_128))
            return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    } else if (U(t->user_data_128) != U(e->user_data_128)) {
        return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    }
    if (t->user_data_64 == 0) {
        if (e->user_data_64 != p->user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    } else if (t->user_data_64 != e->user_data_64) {
        return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    }
    if (t->user_data_32 == 0) {
        if (e->user_data_32 != p->user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    } else if (t->user_data_32 != e->user_data_32) {
        return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    }
    if (t->ledger != 0 && t->ledger != e->ledger) return TB_CT_EXISTS_WITH_DIFFERENT_LEDGER;
    if (t->code != 0 && t->code != e->code) return TB_CT_EXISTS_WITH_DIFFERENT_CODE;
    *ts = e->timestamp;
    return TB_CT_EXISTS;
}

static uint32_t create_transfer_exists(tbo_ctx* c, const tb_transfer_t* t,
                                       const tb_transfer_t* e, uint64_t* ts) {
    if (t->flags != e->flags) return TB_CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (U(t->pending_id) != U(e->pending_id)) return TB_CT_EXISTS_WITH_DIFFERENT_PENDING_ID;
    if (t->timeout != e->timeout) return TB_CT_EXISTS_WITH_DIFFERENT_TIMEOUT;

    if (t->flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
        uint64_t pi = 0;
        int found = get_transfer(c, U(t->pending_id), &pi);
        if (found != 1) abort(); /* the reference asserts the pending transfer exists */
        return post_or_void_pending_transfer_exists(t, e, &c->transfers[pi], ts);
    }
    if (U(t->debit_account_id) != U(e->debit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (U(t->credit_account_id) != U(e->credit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t->flags & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT)) {
        if (U(t->amount) < U(e->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    } else {
        if (U(t->amount) != U(e->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    }
    if (U(t->user_data_128) != U(e->user_data_128))
        return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (t->user_data_64 != e->user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (t->user_data_32 != e->user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (t->ledger != e->ledger) return TB_CT_EXISTS_WITH_DIFFERENT_LEDGER;
    if (t->code != e->code) return TB_CT_EXISTS_WITH_DIFFERENT_CODE;
    *ts = e->timestamp;
    return TB_CT_EXISTS;
}

static uint32_t post_or_void_pending_transfer(tbo_ctx* c, uint64_t timestamp_event,
                                              const tb_transfer_t* t, uint64_t* ts) {
    const uint16_t f = t->flags;
    if ((f & TB_TRANSFER_POST_PENDING) && (f & TB_TRANSFER_VOID_PENDING))
        return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & (TB_TRANSFER_PENDING | TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT |
             TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT))
        return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;

    u128 pending_id = U(t->pending_id);
    if (pending_id == 0) return TB_CT_PENDING_ID_MUST_NOT_BE_ZERO;
    if (pending_id == U128_MAX) return TB_CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
    if (pending_id == U(t->id)) return TB_CT_PENDING_ID_MUST_BE_DIFFERENT;
    if (t->timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;

    uint64_t pi = 0;
    if (get_transfer(c, pending_id, &pi) != 1) return TB_CT_PENDING_TRANSFER_NOT_FOUND;
    const tb_transfer_t p = c->transfers[pi]; /* copy: inserts below may realloc */
    if (!(p.flags & TB_TRANSFER_PENDING)) return TB_CT_PENDING_TRANSFER_NOT_PENDING;

    tb_account_t* dr = get_account(c, U(p.debit_account_id));
    tb_account_t* cr = get_account(c, U(p.credit_account_id));
    if (!dr || !cr) abort(); /* asserted by the reference */

    if (U(t->debit_account_id) > 0 && U(t->debit_account_id) != U(p.debit_account_id))
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (U(t->credit_account_id) > 0 && U(t->credit_account_id) != U(p.credit_account_id))
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t->ledger > 0 && t->ledger != p.ledger) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
    if (t->code > 0 && t->code != p.code) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE;

    u128 amount_actual;
    if (f & TB_TRANSFER_VOID_PENDING) {
        amount_actual = U(t->amount) == 0 ? U(p.amount) : U(t->amount);
    } else {
        amount_actual = U(t->amount) == U128_MAX ? U(p.amount) : U(t->amount);
    }
    if (amount_actual > U(p.amount)) return TB_CT_EXCEEDS_PENDING_TRANSFER_AMOUNT;
    if ((f & TB_TRANSFER_VOID_PENDING) && amount_actual < U(p.amount))
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;

    switch (c->pending_status[pi]) {
        case TB_PENDING_PENDING: break;
        case TB_PENDING_POSTED: return TB_CT_PENDING_TRANSFER_ALREADY_POSTED;
        case TB_PENDING_VOIDED: return TB_CT_PENDING_TRANSFER_ALREADY_VOIDED;
        case TB_PENDING_EXPIRED: return TB_CT_PENDING_TRANSFER_EXPIRED;
        default: abort();
    }

    int has_expiry = p.timeout != 0;
    uint64_t expires_at = 0;
    if (has_expiry) {
        expires_at = p.timestamp + (uint64_t)p.timeout * TB_NS_PER_S;
        if (expires_at <= timestamp_event) return TB_CT_PENDING_TRANSFER_EXPIRED;
    }

    uint64_t timestamp_actual = timestamp_event;
    if (f & TB_TRANSFER_IMPORTED) {
        if (c->transfers_range.has && t->timestamp <= c->transfers_range.key_max)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (map_get(&c->account_by_ts, t->timestamp, NULL))
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        timestamp_actual = t->timestamp;
    }

    if ((dr->flags & TB_ACCOUNT_CLOSED) && !(f & TB_TRANSFER_VOID_PENDING))
        return TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED;
    if ((cr->flags & TB_ACCOUNT_CLOSED) && !(f & TB_TRANSFER_VOID_PENDING))
        return TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED;

    tb_transfer_t row;
    memset(&row, 0, sizeof(row));
    row.id = t->id;
    row.debit_account_id = p.debit_account_id;
    row.credit_account_id = p.credit_account_id;
    row.user_data_128 = U(t->user_data_128) > 0 ? t->user_data_128 : p.user_data_128;
    row.user_data_64 = t->user_data_64 > 0 ? t->user_data_64 : p.user_data_64;
    row.user_data_32 = t->user_data_32 > 0 ? t->user_data_32 : p.user_data_32;
    row.ledger = p.ledger;
    row.code = p.code;
    row.pending_id = t->pending_id;
    row.timeout = 0;
    row.timestamp = timestamp_actual;
    row.flags = t->flags;
    row.amount = W(amount_actual);
    /* dr/cr pointers stay valid: insert_transfer does not touch the accounts array. */
    insert_transfer(c, &row, TB_PENDING_NONE);

    if (has_expiry) {
        /* The expires_at index entry is removed (status below); reset the pulse flag. */
        if (c->pnt_sharded) pnt_log(c, timestamp_actual, expires_at | TBO_PNT_RESET);
        else if (c->pulse_next_timestamp == expires_at) c->pulse_next_timestamp = TB_TIMESTAMP_MIN;
    }
    update_pending_status(c, pi, (f & TB_TRANSFER_POST_PENDING) ? TB_PENDING_POSTED
                                                                 : TB_PENDING_VOIDED);

    tb_account_t dr_new = *dr, cr_new = *cr;
    dr_new.debits_pending = W(U(dr_new.debits_pending) - U(p.amount));
    cr_new.credits_pending = W(U(cr_new.credits_pending) - U(p.amount));
    if (f & TB_TRANSFER_POST_PENDING) {
        dr_new.debits_posted = W(U(dr_new.debits_posted) + amount_actual);
        cr_new.credits_posted = W(U(cr_new.credits_posted) + amount_actual);
    }
    if (f & TB_TRANSFER_VOID_PENDING) {
        if (p.flags & TB_TRANSFER_CLOSING_DEBIT) dr_new.flags &= (uint16_t)~TB_ACCOUNT_CLOSED;
        if (p.flags & TB_TRANSFER_CLOSING_CREDIT) cr_new.flags &= (uint16_t)~TB_ACCOUNT_CLOSED;
    }
    if (amount_actual > 0 || U(p.amount) > 0 || dr_new.flags != dr->flags)
        update_account(c, dr, &dr_new);
    if (amount_actual > 0 || U(p.amount) > 0 || cr_new.flags != cr->flags)
        update_account(c, cr, &cr_new);
    account_event(c, timestamp_actual, &dr_new, &cr_new, t->flags,
                  (f & TB_TRANSFER_POST_PENDING) ? TB_PENDING_POSTED : TB_PENDING_VOIDED, &p,
                  U(t->amount), amount_actual);

    c->commit_timestamp = timestamp_actual;
    *ts = timestamp_actual;
    return TB_STATUS_CREATED;
}

static uint32_t create_transfer(tbo_ctx* c, uint64_t timestamp_event, const tb_transfer_t* t,
                                uint64_t* ts) {
    const uint16_t f = t->flags;
    if (f & TB_TRANSFER_PADDING_MASK) return TB_CT_RESERVED_FLAG;
    u128 id = U(t->id);
    if (id == 0) return TB_CT_ID_MUST_NOT_BE_ZERO;
    if (id == U128_MAX) return TB_CT_ID_MUST_NOT_BE_INT_MAX;

    uint64_t ei = 0;
    switch (get_transfer(c, id, &ei)) {
        case 1: {
            const tb_transfer_t e = c->transfers[ei];
            return create_transfer_exists(c, t, &e, ts);
        }
        case 2: return TB_CT_ID_ALREADY_FAILED;
        default: break;
    }

    if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))
        return post_or_void_pending_transfer(c, timestamp_event, t, ts);

    u128 dr_id = U(t->debit_account_id), cr_id = U(t->credit_account_id);
    if (dr_id == 0) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (dr_id == U128_MAX) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (cr_id == 0) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (cr_id == U128_MAX) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (cr_id == dr_id) return TB_CT_ACCOUNTS_MUST_BE_DIFFERENT;

    if (U(t->pending_id) != 0) return TB_CT_PENDING_ID_MUST_BE_ZERO;
    if (!(f & TB_TRANSFER_PENDING)) {
        if (t->timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
        if (f & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT))
            return TB_CT_CLOSING_TRANSFER_MUST_BE_PENDING;
    }
    if (t->ledger == 0) return TB_CT_LEDGER_MUST_NOT_BE_ZERO;
    if (t->code == 0) return TB_CT_CODE_MUST_NOT_BE_ZERO;

    tb_account_t* dr = get_account(c, dr_id);
    if (!dr) return TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
    tb_account_t* cr = get_account(c, cr_id);
    if (!cr) return TB_CT_CREDIT_ACCOUNT_NOT_FOUND;

    if (dr->ledger != cr->ledger) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t->ledger != dr->ledger) return TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;

    uint64_t timestamp_actual = timestamp_event;
    if (f & TB_TRANSFER_IMPORTED) {
        if (c->transfers_range.has && t->timestamp <= c->transfers_range.key_max)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (map_get(&c->account_by_ts, t->timestamp, NULL))
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (t->timestamp <= dr->timestamp)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_POSTDATE_DEBIT_ACCOUNT;
        if (t->timestamp <= cr->timestamp)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_POSTDATE_CREDIT_ACCOUNT;
        if (t->timeout != 0) return TB_CT_IMPORTED_EVENT_TIMEOUT_MUST_BE_ZERO;
        timestamp_actual = t->timestamp;
    }

    if (dr->flags & TB_ACCOUNT_CLOSED) return TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED;
    if (cr->flags & TB_ACCOUNT_CLOSED) return TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED;

    u128 amount = U(t->amount);
    if (f & TB_TRANSFER_BALANCING_DEBIT) {
        u128 dr_balance = U(dr->debits_posted) + U(dr->debits_pending);
        u128 cp = U(dr->credits_posted);
        u128 room = cp > dr_balance ? cp - dr_balance : 0; /* -| */
        if (room < amount) amount = room;
    }
    if (f & TB_TRANSFER_BALANCING_CREDIT) {
        u128 cr_balance = U(cr->credits_posted) + U(cr->credits_pending);
        u128 dp = U(cr->debits_posted);
        u128 room = dp > cr_balance ? dp - cr_balance : 0;
        if (room < amount) amount = room;
    }

    if (f & TB_TRANSFER_PENDING) {
        if (sum_overflows_u128(amount, U(dr->debits_pending))) return TB_CT_OVERFLOWS_DEBITS_PENDING;
        if (sum_overflows_u128(amount, U(cr->credits_pending)))
            return TB_CT_OVERFLOWS_CREDITS_PENDING;
    }
    if (sum_overflows_u128(amount, U(dr->debits_posted))) return TB_CT_OVERFLOWS_DEBITS_POSTED;
    if (sum_overflows_u128(amount, U(cr->credits_posted))) return TB_CT_OVERFLOWS_CREDITS_POSTED;
    if (sum_overflows_u128(amount, U(dr->debits_pending) + U(dr->debits_posted)))
        return TB_CT_OVERFLOWS_DEBITS;
    if (sum_overflows_u128(amount, U(cr->credits_pending) + U(cr->credits_posted)))
        return TB_CT_OVERFLOWS_CREDITS;
    /* u63 overflow of timestamp + timeout * 1e9 (the product always fits u63). */
    if (timestamp_actual + (uint64_t)t->timeout * TB_NS_PER_S > TB_TIMESTAMP_MAX)
        return TB_CT_OVERFLOWS_TIMEOUT;

    if ((dr->flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
        U(dr->debits_pending) + U(dr->debits_posted) + amount > U(dr->credits_posted))
        return TB_CT_EXCEEDS_CREDITS;
    if ((cr->flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) &&
        U(cr->credits_pending) + U(cr->credits_posted) + amount > U(cr->debits_posted))
        return TB_CT_EXCEEDS_DEBITS;

    tb_transfer_t row = *t;
    row.amount = W(amount);
    row.timestamp = timestamp_actual;
    insert_transfer(c, &row, (f & TB_TRANSFER_PENDING) ? TB_PENDING_PENDING : TB_PENDING_NONE);

    tb_account_t dr_new = *dr, cr_new = *cr;
    if (f & TB_TRANSFER_PENDING) {
        dr_new.debits_pending = W(U(dr_new.debits_pending) + amount);
        cr_new.credits_pending = W(U(cr_new.credits_pending) + amount);
    } else {
        dr_new.debits_posted = W(U(dr_new.debits_posted) + amount);
        cr_new.credits_posted = W(U(cr_new.credits_posted) + amount);
    }
    if (f & TB_TRANSFER_CLOSING_DEBIT) dr_new.flags |= TB_ACCOUNT_CLOSED;
    if (f & TB_TRANSFER_CLOSING_CREDIT) cr_new.flags |= TB_ACCOUNT_CLOSED;
    if (amount > 0 || (dr_new.flags & TB_ACCOUNT_CLOSED)) update_account(c, dr, &dr_new);
    if (amount > 0 || (cr_new.flags & TB_ACCOUNT_CLOSED)) update_account(c, cr, &cr_new);
    account_event(c, timestamp_actual, &dr_new, &cr_new, t->flags,
                  (f & TB_TRANSFER_PENDING) ? TB_PENDING_PENDING : TB_PENDING_NONE, NULL,
                  U(t->amount), amount);

    if (t->timeout > 0) {
        uint64_t expires_at = timestamp_actual + (uint64_t)t->timeout * TB_NS_PER_S;
        if (c->pnt_sharded) pnt_log(c, timestamp_actual, expires_at);
        if (expires_at < c->pulse_next_timestamp) c->pulse_next_timestamp = expires_at;
    }
    c->commit_timestamp = timestamp_actual;
    *ts = timestamp_actual;
    return TB_STATUS_CREATED;
}

/* ---- execute_create (state_machine.zig:3002-3213) ------------------------------------------*/

/* `stamps` (test instrumentation for sharded calls, NULL in the reference's form): event i is
 * stamped stamps[i] instead of timestamp - n + i + 1 -- a shard's part of a linked chain that spans
 * shards keeps its events' global timestamps. `one_chain`: the batch is one linked chain closed at
 * its last event, whatever the events' linked flags (tbg.h TBG_ONE_CHAIN). */
static void execute_create(tbo_ctx* c, int is_transfers, const void* events_, uint32_t n,
                           uint64_t timestamp, const uint64_t* stamps, int one_chain,
                           tb_create_result_t* results) {
    const tb_account_t* accounts = (const tb_account_t*)events_;
    const tb_transfer_t* transfers = (const tb_transfer_t*)events_;
    int64_t chain = -1;
    int chain_broken = 0;
    uint16_t imported_flag = is_transfers ? TB_TRANSFER_IMPORTED : TB_ACCOUNT_IMPORTED;
    uint16_t linked_flag = is_transfers ? TB_TRANSFER_LINKED : TB_ACCOUNT_LINKED;
    int batch_imported = n > 0 && ((is_transfers ? transfers[0].flags : accounts[0].flags) &
                                   imported_flag) != 0;

    for (uint32_t index = 0; index < n; index++) {
        uint16_t flags = is_transfers ? transfers[index].flags : accounts[index].flags;
        uint64_t ev_ts = is_transfers ? transfers[index].timestamp : accounts[index].timestamp;
        const uint64_t timestamp_event = stamps ? stamps[index] : timestamp - n + index + 1;
        uint32_t status;
        uint64_t timestamp_actual = timestamp_event;

        const int linked = one_chain || (flags & linked_flag);
        do {
            if (linked) {
                if (chain < 0) {
                    chain = index;
                    scope_open(c);
                }
                if (index == n - 1 && !one_chain) {
                    status = TB_CT_LINKED_EVENT_CHAIN_OPEN; /* same value for accounts */
                    break;
                }
            }
            if (chain_broken) {
                status = TB_CT_LINKED_EVENT_FAILED;
                break;
            }
            int imported = (flags & imported_flag) != 0;
            if (batch_imported != imported) {
                if (is_transfers)
                    status = imported ? TB_CT_IMPORTED_EVENT_NOT_EXPECTED
                                      : TB_CT_IMPORTED_EVENT_EXPECTED;
                else
                    status = imported ? TB_CA_IMPORTED_EVENT_NOT_EXPECTED
                                      : TB_CA_IMPORTED_EVENT_EXPECTED;
                break;
            }
            if (imported) {
                if (ev_ts < TB_TIMESTAMP_MIN || ev_ts > TB_TIMESTAMP_MAX) {
                    status = is_transfers ? TB_CT_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE
                                          : TB_CA_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE;
                    break;
                }
                if (ev_ts >= timestamp) {
                    status = is_transfers ? TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_ADVANCE
                                          : TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_ADVANCE;
                    break;
                }
            } else if (ev_ts != 0) {
                status = TB_CT_TIMESTAMP_MUST_BE_ZERO; /* same value for accounts */
                break;
            }
            uint64_t ts = timestamp_event;
            status = is_transfers ? create_transfer(c, timestamp_event, &transfers[index], &ts)
                                  : create_account(c, timestamp_event, &accounts[index], &ts);
            /* .created and .exists carry the object's timestamp (state_machine.zig:3098-3104). */
            int exists = is_transfers ? status == TB_CT_EXISTS : status == TB_CA_EXISTS;
            if (status == TB_STATUS_CREATED || exists) timestamp_actual = ts;
        } while (0);

        if (status != TB_STATUS_CREATED) {
            if (chain >= 0) {
                if (!chain_broken) {
                    chain_broken = 1;
                    scope_close(c, 1);
                    for (int64_t ci = chain; ci < index; ci++)
                        results[ci].status = TB_CT_LINKED_EVENT_FAILED;
                }
            }
            /* transient_error: orphan the id (outside any scope). */
            if (is_transfers && tb_transfer_status_transient(status)) {
                map_put(&c->transfer_by_id, U(transfers[index].id), ORPHAN);
            }
        }
        results[index].timestamp = timestamp_actual;
        results[index].status = status;
        results[index].reserved = 0;

        if (chain >= 0 && (!linked || status == TB_CT_LINKED_EVENT_CHAIN_OPEN ||
                           (one_chain && index == n - 1))) {
            if (!chain_broken) scope_close(c, 0);
            chain = -1;
            chain_broken = 0;
        }
    }
}

void tbo_create_accounts(tbo_ctx* c, const tb_account_t* events, uint32_t n, uint64_t timestamp,
                         tb_create_result_t* results) {
    execute_create(c, 0, events, n, timestamp, NULL, 0, results);
}

void tbo_create_transfers(tbo_ctx* c, const tb_transfer_t* events, uint32_t n,
                          uint64_t timestamp, tb_create_result_t* results) {
    if (c->pnt_sharded) c->n_pnt = 0; /* tbo_pnt_ops: this call's updates (tbg_pnt_ops' contract) */
    execute_create(c, 1, events, n, timestamp, NULL, 0, results);
}

/* tbg_create_*'s multi-batch form: batch b holds lens[b] events, stamped as execute_create stamps
 * them with timestamp batch_ts[b]; a sharded call's pulse_next_timestamp log covers the call. */
void tbo_create_accounts_batches(tbo_ctx* c, const tb_account_t* events, const uint32_t* lens,
                                 const uint64_t* batch_ts, uint32_t nb,
                                 tb_create_result_t* results) {
    uint64_t off = 0;
    for (uint32_t b = 0; b < nb; b++) {
        execute_create(c, 0, events + off, lens[b], batch_ts[b], NULL, 0, results + off);
        off += lens[b];
    }
}

void tbo_create_transfers_batches(tbo_ctx* c, const tb_transfer_t* events, const uint32_t* lens,
                                  const uint64_t* batch_ts, uint32_t nb,
                                  tb_create_result_t* results) {
    if (c->pnt_sharded) c->n_pnt = 0;
    uint64_t off = 0;
    for (uint32_t b = 0; b < nb; b++) {
        execute_create(c, 1, events + off, lens[b], batch_ts[b], NULL, 0, results + off);
        off += lens[b];
    }
}

/* Test instrumentation for sharded calls (tbg_create_*_stamped, tbg_forget_orphans,
 * tbg_timestamps_exist in include/tbg.h): per-event timestamps; `timestamp` is the batch's. */
void tbo_create_accounts_stamped(tbo_ctx* c, const tb_account_t* events, uint32_t n,
                                 const uint64_t* stamps, uint64_t timestamp, uint32_t options,
                                 tb_create_result_t* results) {
    execute_create(c, 0, events, n, timestamp ? timestamp : (n ? stamps[n - 1] : 0), stamps,
                   (options & 1) != 0, results);
}

void tbo_create_transfers_stamped(tbo_ctx* c, const tb_transfer_t* events, uint32_t n,
                                  const uint64_t* stamps, uint64_t timestamp, uint32_t options,
                                  tb_create_result_t* results) {
    if (c->pnt_sharded) c->n_pnt = 0;
    execute_create(c, 1, events, n, timestamp ? timestamp : (n ? stamps[n - 1] : 0), stamps,
                   (options & 1) != 0, results);
}

void tbo_key_max(const tbo_ctx* c, uint64_t* accounts_key_max, uint64_t* transfers_key_max) {
    *accounts_key_max = c->accounts_range.has ? c->accounts_range.key_max : 0;
    *transfers_key_max = c->transfers_range.has ? c->transfers_range.key_max : 0;
}

uint64_t tbo_forget_orphans(tbo_ctx* c, const tb_uint128_t* ids, uint32_t n) {
    uint64_t forgotten = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t v;
        if (map_get(&c->transfer_by_id, U(ids[i]), &v) && v == ORPHAN) {
            map_del(&c->transfer_by_id, U(ids[i]));
            forgotten++;
        }
    }
    return forgotten;
}

uint64_t tbo_timestamps_exist(const tbo_ctx* c, int transfers, const uint64_t* ts, uint32_t n,
                              uint8_t* out) {
    uint64_t found = 0;
    for (uint32_t i = 0; i < n; i++) {
        out[i] = (uint8_t)map_get(transfers ? &c->transfer_by_ts : &c->account_by_ts, ts[i], NULL);
        found += out[i];
    }
    return found;
}

/* ---- pulse ----------------------------------------------------------------------------------*/

typedef struct {
    uint64_t expires_at, timestamp, index;
} expiry_key_t;

static int expiry_cmp(const void* a_, const void* b_) {
    const expiry_key_t* a = (const expiry_key_t*)a_;
    const expiry_key_t* b = (const expiry_key_t*)b_;
    if (a->expires_at != b->expires_at) return a->expires_at < b->expires_at ? -1 : 1;
    if (a->timestamp != b->timestamp) return a->timestamp < b->timestamp ? -1 : 1;
    return 0;
}

/* The expires_at index in (expires_at, timestamp) order: pending-status transfers with
 * timeout > 0 (state_machine.zig:443-450); compacts the list. The caller frees *out. */
static uint64_t expiry_sorted(tbo_ctx* c, expiry_key_t** out) {
    expiry_key_t* keys = (expiry_key_t*)xrealloc(NULL, (c->n_expiry + 1) * sizeof(expiry_key_t));
    uint64_t n_keys = 0, w = 0;
    for (uint64_t k = 0; k < c->n_expiry; k++) {
        uint64_t i = c->expiry[k];
        if (c->pending_status[i] != TB_PENDING_PENDING) continue; /* removed from the index */
        c->expiry[w++] = i;                                        /* compact the list */
        const tb_transfer_t* p = &c->transfers[i];
        keys[n_keys].expires_at = p->timestamp + (uint64_t)p->timeout * TB_NS_PER_S;
        keys[n_keys].timestamp = p->timestamp;
        keys[n_keys].index = i;
        n_keys++;
    }
    c->n_expiry = w;
    qsort(keys, n_keys, sizeof(expiry_key_t), expiry_cmp);
    *out = keys;
    return n_keys;
}

/* execute_expire_pending_transfers (:4540-4626) for the first `expired` keys; expiry k is stamped
 * timestamp - expired + k + 1 (:4546), or stamps[k] (a shard's expiries stamped by their positions
 * in the pulse over all shards). */
static void expire_keys(tbo_ctx* c, const expiry_key_t* keys, uint64_t expired, uint64_t timestamp,
                        const uint64_t* stamps) {
    for (uint64_t k = 0; k < expired; k++) {
        const tb_transfer_t* p = &c->transfers[keys[k].index];
        tb_account_t* dr = get_account(c, U(p->debit_account_id));
        tb_account_t* cr = get_account(c, U(p->credit_account_id));
        if (!dr || !cr) abort();
        tb_account_t dr_new = *dr, cr_new = *cr;
        dr_new.debits_pending = W(U(dr_new.debits_pending) - U(p->amount));
        cr_new.credits_pending = W(U(cr_new.credits_pending) - U(p->amount));
        if (p->flags & TB_TRANSFER_CLOSING_DEBIT) dr_new.flags &= (uint16_t)~TB_ACCOUNT_CLOSED;
        if (p->flags & TB_TRANSFER_CLOSING_CREDIT) cr_new.flags &= (uint16_t)~TB_ACCOUNT_CLOSED;
        *dr = dr_new;
        *cr = cr_new;
        c->pending_status[keys[k].index] = TB_PENDING_EXPIRED;
        c->commit_timestamp = stamps ? stamps[k] : timestamp - expired + k + 1;
        account_event(c, c->commit_timestamp, &dr_new, &cr_new, 0, TB_PENDING_EXPIRED, p, 0,
                      U(p->amount));
    }
}

uint32_t tbo_pulse(tbo_ctx* c, uint64_t timestamp) {
    expiry_key_t* keys;
    const uint64_t n_keys = expiry_sorted(c, &keys);
    uint64_t expired = 0;
    while (expired < n_keys && expired < c->pulse_batch_max &&
           keys[expired].expires_at <= timestamp)
        expired++;

    /* ExpirePendingTransfers.finish: buffer_finished iff the buffer filled up. */
    if (expired == c->pulse_batch_max) {
        c->pulse_next_timestamp = keys[expired - 1].expires_at;
    } else if (expired < n_keys) {
        c->pulse_next_timestamp = keys[expired].expires_at; /* first unexpired */
    } else {
        c->pulse_next_timestamp = TB_TIMESTAMP_MAX;
    }
    expire_keys(c, keys, expired, timestamp, NULL);
    free(keys);
    return (uint32_t)expired;
}

uint64_t tbo_pulse_candidates(tbo_ctx* c, uint64_t timestamp, uint64_t* expires_at,
                              uint64_t* timestamps, uint32_t max) {
    expiry_key_t* keys;
    const uint64_t n_keys = expiry_sorted(c, &keys);
    uint64_t n = 0;
    while (n < n_keys && keys[n].expires_at <= timestamp) {
        if (n < max) {
            expires_at[n] = keys[n].expires_at;
            timestamps[n] = keys[n].timestamp;
        }
        n++;
    }
    free(keys);
    return n;
}

uint32_t tbo_pulse_cut(tbo_ctx* c, uint64_t timestamp, uint64_t cut_expires_at,
                       uint64_t cut_timestamp, uint64_t pulse_next_timestamp,
                       const uint64_t* stamps) {
    expiry_key_t* keys;
    const uint64_t n_keys = expiry_sorted(c, &keys);
    uint64_t expired = 0;
    while (expired < n_keys && keys[expired].expires_at <= timestamp &&
           (keys[expired].expires_at < cut_expires_at ||
            (keys[expired].expires_at == cut_expires_at && keys[expired].timestamp <= cut_timestamp)))
        expired++;
    if (pulse_next_timestamp == 0) /* this shard's first unexpired (tbg_pulse_cut's rule) */
        pulse_next_timestamp = expired < n_keys ? keys[expired].expires_at : TB_TIMESTAMP_MAX;
    c->pulse_next_timestamp = pulse_next_timestamp;
    expire_keys(c, keys, expired, timestamp, stamps);
    free(keys);
    return (uint32_t)expired;
}

int tbo_pulse_needed(const tbo_ctx* c, uint64_t timestamp) {
    return c->pulse_next_timestamp <= timestamp;
}

uint64_t tbo_pulse_next_timestamp(const tbo_ctx* c) { return c->pulse_next_timestamp; }

/* ---- lookups / dumps ------------------------------------------------------------------------*/

uint32_t tbo_lookup_accounts(const tbo_ctx* c, const tb_uint128_t* ids, uint32_t n,
                             tb_account_t* out) {
    uint32_t count = 0;
    for (uint32_t k = 0; k < n; k++) {
        uint64_t v;
        if (map_get(&c->account_by_id, U(ids[k]), &v)) out[count++] = c->accounts[v];
    }
    return count;
}

uint32_t tbo_lookup_transfers(const tbo_ctx* c, const tb_uint128_t* ids, uint32_t n,
                              tb_transfer_t* out) {
    uint32_t count = 0;
    for (uint32_t k = 0; k < n; k++) {
        uint64_t v;
        if (map_get(&c->transfer_by_id, U(ids[k]), &v) && v != ORPHAN)
            out[count++] = c->transfers[v];
    }
    return count;
}

int tbo_set_account_balances(tbo_ctx* c, tb_uint128_t id, tb_uint128_t debits_pending,
                             tb_uint128_t debits_posted, tb_uint128_t credits_pending,
                             tb_uint128_t credits_posted) {
    tb_account_t* a = get_account(c, U(id));
    if (!a) return -1;
    a->debits_pending = debits_pending;
    a->debits_posted = debits_posted;
    a->credits_pending = credits_pending;
    a->credits_posted = credits_posted;
    return 0;
}

uint64_t tbo_account_count(const tbo_ctx* c) { return c->n_accounts; }
uint64_t tbo_transfer_count(const tbo_ctx* c) { return c->n_transfers; }

uint64_t tbo_dump_accounts(const tbo_ctx* c, tb_account_t* out) {
    if (out) memcpy(out, c->accounts, c->n_accounts * sizeof(tb_account_t));
    return c->n_accounts;
}
uint64_t tbo_dump_transfers(const tbo_ctx* c, tb_transfer_t* out) {
    if (out) memcpy(out, c->transfers, c->n_transfers * sizeof(tb_transfer_t));
    return c->n_transfers;
}
uint64_t tbo_dump_pending_status(const tbo_ctx* c, uint8_t* out) {
    if (out) memcpy(out, c->pending_status, c->n_transfers);
    return c->n_transfers;
}

void tbo_raise_key_max(tbo_ctx* c, uint64_t accounts_key_max, uint64_t transfers_key_max) {
    if (accounts_key_max) key_range_update(&c->accounts_range, accounts_key_max);
    if (transfers_key_max) key_range_update(&c->transfers_range, transfers_key_max);
}

uint64_t tbo_dump_account_events(const tbo_ctx* c, tb_account_event_t* out) {
    if (out) memcpy(out, c->events, c->n_events * sizeof(tb_account_event_t));
    return c->n_events;
}

/* ---- get_change_events (state_machine.zig:2396-2434 filter, :3395-3527 execution) -----------*/

static const tbo_ctx* g_sort_ctx;
static int event_index_cmp(const void* a_, const void* b_) {
    const uint64_t a = *(const uint64_t*)a_, b = *(const uint64_t*)b_;
    const uint64_t ta = g_sort_ctx->events[a].timestamp, tb = g_sort_ctx->events[b].timestamp;
    if (ta != tb) return ta < tb ? -1 : 1;
    return a < b ? -1 : (a > b);
}

int64_t tbo_get_change_events(const tbo_ctx* c, const tb_change_events_filter_t* filter,
                              uint32_t limit_max, tb_change_event_t* out) {
    /* get_scan_from_change_events_filter: an invalid filter yields no results. */
    int reserved_zero = 1;
    for (int i = 0; i < 44; i++) reserved_zero &= filter->reserved[i] == 0;
    const uint64_t tmin = filter->timestamp_min, tmax = filter->timestamp_max;
    int valid = (tmin == 0 || (tmin >= TB_TIMESTAMP_MIN && tmin <= TB_TIMESTAMP_MAX)) &&
                (tmax == 0 || (tmax >= TB_TIMESTAMP_MIN && tmax <= TB_TIMESTAMP_MAX)) &&
                (tmax == 0 || tmin <= tmax) && filter->limit != 0 && reserved_zero;
    if (!valid) return 0;
    const uint64_t lo = tmin == 0 ? TB_TIMESTAMP_MIN : tmin;
    const uint64_t hi = tmax == 0 ? TB_TIMESTAMP_MAX : tmax;
    const uint32_t limit = filter->limit < limit_max ? filter->limit : limit_max;
    /* The groove is keyed by timestamp: ascending order. */
    uint64_t* order = (uint64_t*)xrealloc(NULL, (c->n_events + 1) * sizeof(uint64_t));
    for (uint64_t i = 0; i < c->n_events; i++) order[i] = i;
    g_sort_ctx = c;
    qsort(order, c->n_events, sizeof(uint64_t), event_index_cmp);
    uint32_t count = 0;
    for (uint64_t j = 0; j < c->n_events && count < limit; j++) {
        const tb_account_event_t* e = &c->events[order[j]];
        if (e->timestamp < lo || e->timestamp > hi) continue;
        uint64_t ti = 0;
        /* get_change_event: the transfer by timestamp, the pending transfer for an expiry. */
        if (e->transfer_pending_status == TB_PENDING_EXPIRED) {
            if (get_transfer((tbo_ctx*)c, U(e->transfer_pending_id), &ti) != 1) abort();
        } else if (!map_get(&c->transfer_by_ts, e->timestamp, &ti)) {
            abort();
        }
        const tb_transfer_t* t = &c->transfers[ti];
        const tb_account_t* dr = get_account((tbo_ctx*)c, U(e->dr_account_id));
        const tb_account_t* cr = get_account((tbo_ctx*)c, U(e->cr_account_id));
        if (!dr || !cr) abort();
        tb_change_event_t* o = &out[count++];
        memset(o, 0, sizeof(*o));
        o->transfer_id = t->id;
        o->transfer_amount = e->amount;
        o->transfer_pending_id = t->pending_id;
        o->transfer_user_data_128 = t->user_data_128;
        o->transfer_user_data_64 = t->user_data_64;
        o->transfer_user_data_32 = t->user_data_32;
        o->transfer_timeout = t->timeout;
        o->ledger = e->ledger;
        o->transfer_code = t->code;
        o->transfer_flags = t->flags;
        switch (e->transfer_pending_status) {
            case TB_PENDING_NONE: o->type = TB_CHANGE_SINGLE_PHASE; break;
            case TB_PENDING_PENDING: o->type = TB_CHANGE_TWO_PHASE_PENDING; break;
            case TB_PENDING_POSTED: o->type = TB_CHANGE_TWO_PHASE_POSTED; break;
            case TB_PENDING_VOIDED: o->type = TB_CHANGE_TWO_PHASE_VOIDED; break;
            default: o->type = TB_CHANGE_TWO_PHASE_EXPIRED; break;
        }
        o->debit_account_id = dr->id;
        o->debit_account_debits_pending = e->dr_debits_pending;
        o->debit_account_debits_posted = e->dr_debits_posted;
        o->debit_account_credits_pending = e->dr_credits_pending;
        o->debit_account_credits_posted = e->dr_credits_posted;
        o->debit_account_user_data_128 = dr->user_data_128;
        o->debit_account_user_data_64 = dr->user_data_64;
        o->debit_account_user_data_32 = dr->user_data_32;
        o->debit_account_code = dr->code;
        o->debit_account_flags = e->dr_account_flags;
        o->credit_account_id = cr->id;
        o->credit_account_debits_pending = e->cr_debits_pending;
        o->credit_account_debits_posted = e->cr_debits_posted;
        o->credit_account_credits_pending = e->cr_credits_pending;
        o->credit_account_credits_posted = e->cr_credits_posted;
        o->credit_account_user_data_128 = cr->user_data_128;
        o->credit_account_user_data_64 = cr->user_data_64;
        o->credit_account_user_data_32 = cr->user_data_32;
        o->credit_account_code = cr->code;
        o->credit_account_flags = e->cr_account_flags;
        o->timestamp = e->timestamp;
        o->transfer_timestamp = t->timestamp;
        o->debit_account_timestamp = dr->timestamp;
        o->credit_account_timestamp = cr->timestamp;
    }
    free(order);
    return count;
}

/* ---- scans: get_account_transfers / get_account_balances / query_* ---------------------------
 * get_scan_from_account_filter (state_machine.zig:1737-1841), get_scan_from_query_filter
 * (:2054-2123), prefetch_get_account_balances_scan (:1608-1675), execute_* (:3294-3393). The
 * grooves' index scans are restated as a walk over the objects in timestamp order (creation order:
 * timestamps only grow, imported ones included), ascending or descending, keeping the objects every
 * nonzero condition matches, up to the limit. */

static int ts_in_range(uint64_t ts) { return ts >= TB_TIMESTAMP_MIN && ts <= TB_TIMESTAMP_MAX; }

static int account_filter_valid(const tb_account_filter_t* f) {
    int reserved_zero = 1;
    for (int i = 0; i < 58; i++) reserved_zero &= f->reserved[i] == 0;
    const u128 id = U(f->account_id);
    return id != 0 && id != U128_MAX && (f->timestamp_min == 0 || ts_in_range(f->timestamp_min)) &&
           (f->timestamp_max == 0 || ts_in_range(f->timestamp_max)) &&
           (f->timestamp_max == 0 || f->timestamp_min <= f->timestamp_max) && f->limit != 0 &&
           (f->flags & (TB_ACCOUNT_FILTER_DEBITS | TB_ACCOUNT_FILTER_CREDITS)) &&
           !(f->flags & TB_ACCOUNT_FILTER_PADDING_MASK) && reserved_zero;
}

static int query_filter_valid(const tb_query_filter_t* f) {
    int reserved_zero = 1;
    for (int i = 0; i < 6; i++) reserved_zero &= f->reserved[i] == 0;
    return (f->timestamp_min == 0 || ts_in_range(f->timestamp_min)) &&
           (f->timestamp_max == 0 || ts_in_range(f->timestamp_max)) &&
           (f->timestamp_max == 0 || f->timestamp_min <= f->timestamp_max) && f->limit != 0 &&
           !(f->flags & TB_QUERY_FILTER_PADDING_MASK) && reserved_zero;
}

static int account_filter_match(const tb_account_filter_t* f, const tb_transfer_t* t) {
    const u128 id = U(f->account_id);
    const int on_side = ((f->flags & TB_ACCOUNT_FILTER_DEBITS) && U(t->debit_account_id) == id) ||
                        ((f->flags & TB_ACCOUNT_FILTER_CREDITS) && U(t->credit_account_id) == id);
    const uint64_t lo = f->timestamp_min ? f->timestamp_min : TB_TIMESTAMP_MIN;
    const uint64_t hi = f->timestamp_max ? f->timestamp_max : TB_TIMESTAMP_MAX;
    return on_side && t->timestamp >= lo && t->timestamp <= hi &&
           (U(f->user_data_128) == 0 || U(f->user_data_128) == U(t->user_data_128)) &&
           (f->user_data_64 == 0 || f->user_data_64 == t->user_data_64) &&
           (f->user_data_32 == 0 || f->user_data_32 == t->user_data_32) &&
           (f->code == 0 || f->code == t->code);
}

#define QUERY_MATCH(f, o)                                                                        \
    ((o)->timestamp >= ((f)->timestamp_min ? (f)->timestamp_min : TB_TIMESTAMP_MIN) &&           \
     (o)->timestamp <= ((f)->timestamp_max ? (f)->timestamp_max : TB_TIMESTAMP_MAX) &&           \
     (U((f)->user_data_128) == 0 || U((f)->user_data_128) == U((o)->user_data_128)) &&           \
     ((f)->user_data_64 == 0 || (f)->user_data_64 == (o)->user_data_64) &&                       \
     ((f)->user_data_32 == 0 || (f)->user_data_32 == (o)->user_data_32) &&                       \
     ((f)->ledger == 0 || (f)->ledger == (o)->ledger) && ((f)->code == 0 || (f)->code == (o)->code))

/* The i-th object of the walk (ascending or descending). */
static uint64_t walk_at(uint64_t n, uint64_t i, int reversed) { return reversed ? n - 1 - i : i; }

int64_t tbo_get_account_transfers(const tbo_ctx* c, const tb_account_filter_t* filter,
                                  uint32_t limit_max, tb_transfer_t* out) {
    if (!account_filter_valid(filter)) return 0;
    const uint32_t limit = filter->limit < limit_max ? filter->limit : limit_max;
    const int rev = (filter->flags & TB_ACCOUNT_FILTER_REVERSED) != 0;
    uint32_t count = 0;
    for (uint64_t i = 0; i < c->n_transfers && count < limit; i++) {
        const tb_transfer_t* t = &c->transfers[walk_at(c->n_transfers, i, rev)];
        if (account_filter_match(filter, t)) out[count++] = *t;
    }
    return count;
}

int64_t tbo_get_account_balances(const tbo_ctx* c, const tb_account_filter_t* filter,
                                 uint32_t limit_max, tb_account_balance_t* out) {
    /* The account must exist and keep history (:1624-1626). */
    const tb_account_t* a = get_account((tbo_ctx*)c, U(filter->account_id));
    if (!a || !(a->flags & TB_ACCOUNT_HISTORY) || !account_filter_valid(filter)) return 0;
    const uint32_t limit = filter->limit < limit_max ? filter->limit : limit_max;
    const int rev = (filter->flags & TB_ACCOUNT_FILTER_REVERSED) != 0;
    const u128 id = U(filter->account_id);
    /* The groove keyed by timestamp (the log sorted, as get_change_events reads it). */
    uint64_t* order = (uint64_t*)xrealloc(NULL, (c->n_events + 1) * sizeof(uint64_t));
    for (uint64_t i = 0; i < c->n_events; i++) order[i] = i;
    g_sort_ctx = c;
    qsort(order, c->n_events, sizeof(uint64_t), event_index_cmp);
    uint32_t count = 0;
    for (uint64_t i = 0; i < c->n_transfers && count < limit; i++) {
        const tb_transfer_t* t = &c->transfers[walk_at(c->n_transfers, i, rev)];
        if (!account_filter_match(filter, t)) continue;
        /* AccountBalancesScanLookup: the AccountEvent with the transfer's timestamp. */
        uint64_t lo = 0, hi = c->n_events;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (c->events[order[mid]].timestamp < t->timestamp) lo = mid + 1;
            else hi = mid;
        }
        if (lo == c->n_events || c->events[order[lo]].timestamp != t->timestamp) abort();
        const tb_account_event_t* e = &c->events[order[lo]];
        tb_account_balance_t* b = &out[count++];
        memset(b, 0, sizeof(*b));
        b->timestamp = e->timestamp;
        if (U(e->dr_account_id) == id) {
            b->debits_pending = e->dr_debits_pending;
            b->debits_posted = e->dr_debits_posted;
            b->credits_pending = e->dr_credits_pending;
            b->credits_posted = e->dr_credits_posted;
        } else if (U(e->cr_account_id) == id) {
            b->debits_pending = e->cr_debits_pending;
            b->debits_posted = e->cr_debits_posted;
            b->credits_pending = e->cr_credits_pending;
            b->credits_posted = e->cr_credits_posted;
        } else {
            abort();
        }
    }
    free(order);
    return count;
}

int64_t tbo_query_accounts(const tbo_ctx* c, const tb_query_filter_t* filter, uint32_t limit_max,
                           tb_account_t* out) {
    if (!query_filter_valid(filter)) return 0;
    const uint32_t limit = filter->limit < limit_max ? filter->limit : limit_max;
    const int rev = (filter->flags & TB_QUERY_FILTER_REVERSED) != 0;
    uint32_t count = 0;
    for (uint64_t i = 0; i < c->n_accounts && count < limit; i++) {
        const tb_account_t* a = &c->accounts[walk_at(c->n_accounts, i, rev)];
        if (QUERY_MATCH(filter, a)) out[count++] = *a;
    }
    return count;
}

int64_t tbo_query_transfers(const tbo_ctx* c, const tb_query_filter_t* filter,
                            uint32_t limit_max, tb_transfer_t* out) {
    if (!query_filter_valid(filter)) return 0;
    const uint32_t limit = filter->limit < limit_max ? filter->limit : limit_max;
    const int rev = (filter->flags & TB_QUERY_FILTER_REVERSED) != 0;
    uint32_t count = 0;
    for (uint64_t i = 0; i < c->n_transfers && count < limit; i++) {
        const tb_transfer_t* t = &c->transfers[walk_at(c->n_transfers, i, rev)];
        if (QUERY_MATCH(filter, t)) out[count++] = *t;
    }
    return count;
}

/* ---- executor binding (tb_state_machine.h) --------------------------------------------------*/

static int ex_create_accounts(void* self, const tb_account_t* events, uint32_t n,
                              const uint32_t* lens, const uint64_t* ts, uint32_t nb,
                              tb_create_result_t* results) {
    uint32_t offset = 0;
    for (uint32_t b = 0; b < nb; b++) {
        tbo_create_accounts((tbo_ctx*)self, events + offset, lens[b], ts[b], results + offset);
        offset += lens[b];
    }
    return offset == n ? 0 : -22;
}
static int ex_create_transfers(void* self, const tb_transfer_t* events, uint32_t n,
                               const uint32_t* lens, const uint64_t* ts, uint32_t nb,
                               tb_create_result_t* results) {
    uint32_t offset = 0;
    for (uint32_t b = 0; b < nb; b++) {
        tbo_create_transfers((tbo_ctx*)self, events + offset, lens[b], ts[b], results + offset);
        offset += lens[b];
    }
    return offset == n ? 0 : -22;
}
static int64_t ex_pulse(void* self, uint64_t ts) { return tbo_pulse((tbo_ctx*)self, ts); }
static uint64_t ex_pulse_next(void* self) { return tbo_pulse_next_timestamp((tbo_ctx*)self); }
static int64_t ex_lookup_accounts(void* self, const tb_uint128_t* ids, uint32_t n,
                                  tb_account_t* out) {
    return tbo_lookup_accounts((tbo_ctx*)self, ids, n, out);
}
static int64_t ex_lookup_transfers(void* self, const tb_uint128_t* ids, uint32_t n,
                                   tb_transfer_t* out) {
    return tbo_lookup_transfers((tbo_ctx*)self, ids, n, out);
}
static int64_t ex_get_change_events(void* self, const tb_change_events_filter_t* filter,
                                    uint32_t limit_max, tb_change_event_t* out) {
    return tbo_get_change_events((tbo_ctx*)self, filter, limit_max, out);
}

static int64_t ex_get_account_transfers(void* self, const tb_account_filter_t* f, uint32_t m,
                                        tb_transfer_t* out) {
    return tbo_get_account_transfers((tbo_ctx*)self, f, m, out);
}
static int64_t ex_get_account_balances(void* self, const tb_account_filter_t* f, uint32_t m,
                                       tb_account_balance_t* out) {
    return tbo_get_account_balances((tbo_ctx*)self, f, m, out);
}
static int64_t ex_query_accounts(void* self, const tb_query_filter_t* f, uint32_t m,
                                 tb_account_t* out) {
    return tbo_query_accounts((tbo_ctx*)self, f, m, out);
}
static int64_t ex_query_transfers(void* self, const tb_query_filter_t* f, uint32_t m,
                                  tb_transfer_t* out) {
    return tbo_query_transfers((tbo_ctx*)self, f, m, out);
}

void tbo_executor_fill(tbo_ctx* c, tb_executor* ex) {
    ex->self = c;
    ex->create_accounts = ex_create_accounts;
    ex->create_transfers = ex_create_transfers;
    ex->pulse = ex_pulse;
    ex->pulse_next_timestamp = ex_pulse_next;
    ex->lookup_accounts = ex_lookup_accounts;
    ex->lookup_transfers = ex_lookup_transfers;
    ex->get_change_events = ex_get_change_events;
    ex->get_account_transfers = ex_get_account_transfers;
    ex->get_account_balances = ex_get_account_balances;
    ex->query_accounts = ex_query_accounts;
    ex->query_transfers = ex_query_transfers;
}

/* ---- the shard executor interface (include/tbg_group.h tbg_shard_ops) ------------------------
 * Test instrumentation: binds this oracle as one shard of a tbg_group_open_shards group, so the
 * group's exact engine (tigerbeetle_amd/csrc/engine.cpp) runs over oracle shards in the CPU tests
 * exactly as it runs over HIP executors. */
static int sh_create_accounts(void* self, const tb_account_t* ev, uint32_t n, const uint32_t* lens,
                              const uint64_t* bts, uint32_t nb, tb_create_result_t* out) {
    (void)n;
    tbo_create_accounts_batches((tbo_ctx*)self, ev, lens, bts, nb, out);
    return 0;
}
static int sh_create_transfers(void* self, const tb_transfer_t* ev, uint32_t n,
                               const uint32_t* lens, const uint64_t* bts, uint32_t nb,
                               tb_create_result_t* out) {
    (void)n;
    tbo_create_transfers_batches((tbo_ctx*)self, ev, lens, bts, nb, out);
    return 0;
}
static int sh_create_accounts_stamped(void* self, const tb_account_t* ev, uint32_t n,
                                      const uint64_t* st, uint64_t bts, uint32_t opt,
                                      tb_create_result_t* out) {
    tbo_create_accounts_stamped((tbo_ctx*)self, ev, n, st, bts, opt, out);
    return 0;
}
static int sh_create_transfers_stamped(void* self, const tb_transfer_t* ev, uint32_t n,
                                       const uint64_t* st, uint64_t bts, uint32_t opt,
                                       tb_create_result_t* out) {
    tbo_create_transfers_stamped((tbo_ctx*)self, ev, n, st, bts, opt, out);
    return 0;
}
static int64_t sh_forget_orphans(void* self, const tb_uint128_t* ids, uint32_t n) {
    return (int64_t)tbo_forget_orphans((tbo_ctx*)self, ids, n);
}
static int64_t sh_timestamps_exist(void* self, int transfers, const uint64_t* ts, uint32_t n,
                                   uint8_t* out) {
    return (int64_t)tbo_timestamps_exist((const tbo_ctx*)self, transfers, ts, n, out);
}
static int sh_key_max(void* self, uint64_t* a, uint64_t* t) {
    tbo_key_max((const tbo_ctx*)self, a, t);
    return 0;
}
static int sh_raise_key_max(void* self, uint64_t a, uint64_t t) {
    tbo_raise_key_max((tbo_ctx*)self, a, t);
    return 0;
}
static int sh_set_pnt_sharded(void* self, int on) {
    tbo_pnt_sharded((tbo_ctx*)self, on);
    return 0;
}
/* tbg_pnt_ops' contract: the count (nothing copied) with ts == NULL; else up to `max` copied. */
static int64_t sh_pnt_ops(void* self, uint64_t* ts, uint64_t* ops, uint64_t max, uint64_t* start) {
    tbo_ctx* c = (tbo_ctx*)self;
    if (!ts || !ops) return (int64_t)tbo_pnt_ops(c, NULL, NULL, start);
    if (c->n_pnt > max) return -22;
    return (int64_t)tbo_pnt_ops(c, ts, ops, start);
}
static uint64_t sh_pulse_next(void* self) { return tbo_pulse_next_timestamp((tbo_ctx*)self); }
static int sh_set_pulse_next(void* self, uint64_t v) {
    tbo_set_pulse_next_timestamp((tbo_ctx*)self, v);
    return 0;
}
static int64_t sh_pulse_candidates(void* self, uint64_t ts, uint64_t* e, uint64_t* t,
                                   uint32_t max) {
    return (int64_t)tbo_pulse_candidates((tbo_ctx*)self, ts, e, t, max);
}
static int64_t sh_pulse_cut(void* self, uint64_t ts, uint64_t ce, uint64_t ct, uint64_t pnt,
                            const uint64_t* stamps) {
    return (int64_t)tbo_pulse_cut((tbo_ctx*)self, ts, ce, ct, pnt, stamps);
}
static int64_t sh_lookup_accounts(void* self, const tb_uint128_t* ids, uint32_t n,
                                  tb_account_t* out) {
    return (int64_t)tbo_lookup_accounts((const tbo_ctx*)self, ids, n, out);
}
static int64_t sh_lookup_transfers(void* self, const tb_uint128_t* ids, uint32_t n,
                                   tb_transfer_t* out) {
    return (int64_t)tbo_lookup_transfers((const tbo_ctx*)self, ids, n, out);
}

void tbo_shard_ops_fill(tbg_shard_ops* ops) {
    ops->create_accounts = sh_create_accounts;
    ops->create_transfers = sh_create_transfers;
    ops->create_accounts_stamped = sh_create_accounts_stamped;
    ops->create_transfers_stamped = sh_create_transfers_stamped;
    ops->forget_orphans = sh_forget_orphans;
    ops->timestamps_exist = sh_timestamps_exist;
    ops->key_max = sh_key_max;
    ops->raise_key_max = sh_raise_key_max;
    ops->set_pnt_sharded = sh_set_pnt_sharded;
    ops->pnt_ops = sh_pnt_ops;
    ops->pulse_next_timestamp = sh_pulse_next;
    ops->set_pulse_next_timestamp = sh_set_pulse_next;
    ops->pulse_candidates = sh_pulse_candidates;
    ops->pulse_cut = sh_pulse_cut;
    ops->lookup_accounts = sh_lookup_accounts;
    ops->lookup_transfers = sh_lookup_transfers;
}
