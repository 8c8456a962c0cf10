/*
 * tb_types.h -- the extern data layouts of TigerBeetle's commit path, bit-identical to the
 * reference (`src/tigerbeetle.zig`), shared by the C-ABI executor (tbg.h), the C++
 * StateMachine mirror (tb_state_machine.h) and the CPU oracle (oracle/tb_oracle.h).
 *
 * u128 fields are carried as two little-endian u64 words {lo, hi}: the in-memory byte image is
 * exactly Zig's little-endian u128, so a buffer produced by the reference client can be handed
 * over as-is.
 *
 * Reference: src/tigerbeetle.zig:10-43 (Account), :45-68 (AccountFlags), :85-116 (Transfer),
 * :132-148 (TransferFlags), :153-215 (CreateAccountStatus), :220-469 (CreateTransferStatus),
 * :471-493 (Create*Result); src/lsm/timestamp_range.zig (timestamp_min/max).
 */
#ifndef TB_TYPES_H
#define TB_TYPES_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tb_uint128 {
    uint64_t lo;
    uint64_t hi;
} tb_uint128_t;

/* src/tigerbeetle.zig:10-43 -- 128 bytes, align 16, no padding. */
typedef struct tb_account {
    tb_uint128_t id;
    tb_uint128_t debits_pending;
    tb_uint128_t debits_posted;
    tb_uint128_t credits_pending;
    tb_uint128_t credits_posted;
    tb_uint128_t user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t reserved;
    uint32_t ledger;
    uint16_t code;
    uint16_t flags;
    uint64_t timestamp;
} tb_account_t;

/* src/tigerbeetle.zig:85-116 -- 128 bytes, align 16, no padding. */
typedef struct tb_transfer {
    tb_uint128_t id;
    tb_uint128_t debit_account_id;
    tb_uint128_t credit_account_id;
    tb_uint128_t amount;
    tb_uint128_t pending_id;
    tb_uint128_t user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t timeout;
    uint32_t ledger;
    uint16_t code;
    uint16_t flags;
    uint64_t timestamp;
} tb_transfer_t;

/* src/tigerbeetle.zig:471-493 -- 16 bytes, align 8. */
typedef struct tb_create_result {
    uint64_t timestamp;
    uint32_t status;
    uint32_t reserved;
} tb_create_result_t;

/* AccountEvent, src/state_machine.zig:104-220 -- 256 bytes, align 16, no padding: one per
 * created transfer, post/void and expiry, with both accounts' balances and flags as they stand
 * after the event (account_event, :4384-4465). The groove `account_events` stores it; CDC reads it
 * back through get_change_events. */
typedef struct tb_account_event {
    tb_uint128_t dr_account_id;
    tb_uint128_t dr_debits_pending;
    tb_uint128_t dr_debits_posted;
    tb_uint128_t dr_credits_pending;
    tb_uint128_t dr_credits_posted;
    tb_uint128_t cr_account_id;
    tb_uint128_t cr_debits_pending;
    tb_uint128_t cr_debits_posted;
    tb_uint128_t cr_credits_pending;
    tb_uint128_t cr_credits_posted;
    uint64_t timestamp;
    uint64_t dr_account_timestamp;
    uint64_t cr_account_timestamp;
    uint16_t dr_account_flags;
    uint16_t cr_account_flags;
    uint16_t transfer_flags;
    uint16_t transfer_pending_flags;
    tb_uint128_t transfer_pending_id;
    tb_uint128_t amount_requested;
    tb_uint128_t amount;
    uint32_t ledger;
    uint8_t transfer_pending_status; /* TB_PENDING_* of the event (expired: an expiry) */
    uint8_t reserved[11];
} tb_account_event_t;

/* ChangeEventType, src/tigerbeetle.zig:614-620. */
enum {
    TB_CHANGE_SINGLE_PHASE = 0,
    TB_CHANGE_TWO_PHASE_PENDING = 1,
    TB_CHANGE_TWO_PHASE_POSTED = 2,
    TB_CHANGE_TWO_PHASE_VOIDED = 3,
    TB_CHANGE_TWO_PHASE_EXPIRED = 4,
};

/* ChangeEvent, src/tigerbeetle.zig:622-670 -- 384 bytes (a transfer + 2 accounts), align 16. */
typedef struct tb_change_event {
    tb_uint128_t transfer_id;
    tb_uint128_t transfer_amount;
    tb_uint128_t transfer_pending_id;
    tb_uint128_t transfer_user_data_128;
    uint64_t transfer_user_data_64;
    uint32_t transfer_user_data_32;
    uint32_t transfer_timeout;
    uint16_t transfer_code;
    uint16_t transfer_flags;
    uint32_t ledger;
    uint8_t type;
    uint8_t reserved[39];
    tb_uint128_t debit_account_id;
    tb_uint128_t debit_account_debits_pending;
    tb_uint128_t debit_account_debits_posted;
    tb_uint128_t debit_account_credits_pending;
    tb_uint128_t debit_account_credits_posted;
    tb_uint128_t debit_account_user_data_128;
    uint64_t debit_account_user_data_64;
    uint32_t debit_account_user_data_32;
    uint16_t debit_account_code;
    uint16_t debit_account_flags;
    tb_uint128_t credit_account_id;
    tb_uint128_t credit_account_debits_pending;
    tb_uint128_t credit_account_debits_posted;
    tb_uint128_t credit_account_credits_pending;
    tb_uint128_t credit_account_credits_posted;
    tb_uint128_t credit_account_user_data_128;
    uint64_t credit_account_user_data_64;
    uint32_t credit_account_user_data_32;
    uint16_t credit_account_code;
    uint16_t credit_account_flags;
    uint64_t timestamp;
    uint64_t transfer_timestamp;
    uint64_t debit_account_timestamp;
    uint64_t credit_account_timestamp;
} tb_change_event_t;

/* ChangeEventsFilter, src/tigerbeetle.zig:672-682 -- 64 bytes. */
typedef struct tb_change_events_filter {
    uint64_t timestamp_min; /* 0: timestamp_min */
    uint64_t timestamp_max; /* 0: timestamp_max */
    uint32_t limit;
    uint8_t reserved[44];
} tb_change_events_filter_t;

/* AccountFilter, src/tigerbeetle.zig:563-611 -- 128 bytes: get_account_transfers and
 * get_account_balances. Zero fields do not filter. */
typedef struct tb_account_filter {
    tb_uint128_t account_id;
    tb_uint128_t user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint16_t code;
    uint8_t reserved[58];
    uint64_t timestamp_min; /* inclusive; 0: timestamp_min */
    uint64_t timestamp_max; /* inclusive; 0: timestamp_max */
    uint32_t limit;
    uint32_t flags;         /* TB_ACCOUNT_FILTER_* */
} tb_account_filter_t;

enum {
    TB_ACCOUNT_FILTER_DEBITS = 1u << 0,
    TB_ACCOUNT_FILTER_CREDITS = 1u << 1,
    TB_ACCOUNT_FILTER_REVERSED = 1u << 2,
    TB_ACCOUNT_FILTER_PADDING_MASK = ~7u,
};

/* QueryFilter, src/tigerbeetle.zig:517-561 -- 64 bytes: query_accounts and query_transfers. */
typedef struct tb_query_filter {
    tb_uint128_t user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t ledger;
    uint16_t code;
    uint8_t reserved[6];
    uint64_t timestamp_min;
    uint64_t timestamp_max;
    uint32_t limit;
    uint32_t flags;         /* TB_QUERY_FILTER_REVERSED */
} tb_query_filter_t;

enum {
    TB_QUERY_FILTER_REVERSED = 1u << 0,
    TB_QUERY_FILTER_PADDING_MASK = ~1u,
};

/* AccountBalance, src/tigerbeetle.zig:70-84 -- 128 bytes: an account's balances as they stood
 * after one of its transfers (get_account_balances). */
typedef struct tb_account_balance {
    tb_uint128_t debits_pending;
    tb_uint128_t debits_posted;
    tb_uint128_t credits_pending;
    tb_uint128_t credits_posted;
    uint64_t timestamp;
    uint8_t reserved[56];
} tb_account_balance_t;

/* AccountFlags, src/tigerbeetle.zig:45-68 (packed struct(u16), LSB first). */
enum {
    TB_ACCOUNT_LINKED = 1u << 0,
    TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS = 1u << 1,
    TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS = 1u << 2,
    TB_ACCOUNT_HISTORY = 1u << 3,
    TB_ACCOUNT_IMPORTED = 1u << 4,
    TB_ACCOUNT_CLOSED = 1u << 5,
    TB_ACCOUNT_PADDING_MASK = 0xFFC0u,
};

/* TransferFlags, src/tigerbeetle.zig:132-148. */
enum {
    TB_TRANSFER_LINKED = 1u << 0,
    TB_TRANSFER_PENDING = 1u << 1,
    TB_TRANSFER_POST_PENDING = 1u << 2,
    TB_TRANSFER_VOID_PENDING = 1u << 3,
    TB_TRANSFER_BALANCING_DEBIT = 1u << 4,
    TB_TRANSFER_BALANCING_CREDIT = 1u << 5,
    TB_TRANSFER_CLOSING_DEBIT = 1u << 6,
    TB_TRANSFER_CLOSING_CREDIT = 1u << 7,
    TB_TRANSFER_IMPORTED = 1u << 8,
    TB_TRANSFER_PADDING_MASK = 0xFE00u,
};

/* TransferPendingStatus, src/tigerbeetle.zig:118-130. */
enum {
    TB_PENDING_NONE = 0,
    TB_PENDING_PENDING = 1,
    TB_PENDING_POSTED = 2,
    TB_PENDING_VOIDED = 3,
    TB_PENDING_EXPIRED = 4,
};

#define TB_STATUS_CREATED 0xFFFFFFFFu

/* CreateAccountStatus, src/tigerbeetle.zig:153-215 (numeric values, NOT precedence order). */
enum {
    TB_CA_LINKED_EVENT_FAILED = 1,
    TB_CA_LINKED_EVENT_CHAIN_OPEN = 2,
    TB_CA_TIMESTAMP_MUST_BE_ZERO = 3,
    TB_CA_RESERVED_FIELD = 4,
    TB_CA_RESERVED_FLAG = 5,
    TB_CA_ID_MUST_NOT_BE_ZERO = 6,
    TB_CA_ID_MUST_NOT_BE_INT_MAX = 7,
    TB_CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 8,
    TB_CA_DEBITS_PENDING_MUST_BE_ZERO = 9,
    TB_CA_DEBITS_POSTED_MUST_BE_ZERO = 10,
    TB_CA_CREDITS_PENDING_MUST_BE_ZERO = 11,
    TB_CA_CREDITS_POSTED_MUST_BE_ZERO = 12,
    TB_CA_LEDGER_MUST_NOT_BE_ZERO = 13,
    TB_CA_CODE_MUST_NOT_BE_ZERO = 14,
    TB_CA_EXISTS_WITH_DIFFERENT_FLAGS = 15,
    TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 16,
    TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 17,
    TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 18,
    TB_CA_EXISTS_WITH_DIFFERENT_LEDGER = 19,
    TB_CA_EXISTS_WITH_DIFFERENT_CODE = 20,
    TB_CA_EXISTS = 21,
    TB_CA_IMPORTED_EVENT_EXPECTED = 22,
    TB_CA_IMPORTED_EVENT_NOT_EXPECTED = 23,
    TB_CA_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE = 24,
    TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_ADVANCE = 25,
    TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS = 26,
};

/* CreateTransferStatus, src/tigerbeetle.zig:220-320. */
enum {
    TB_CT_LINKED_EVENT_FAILED = 1,
    TB_CT_LINKED_EVENT_CHAIN_OPEN = 2,
    TB_CT_TIMESTAMP_MUST_BE_ZERO = 3,
    TB_CT_RESERVED_FLAG = 4,
    TB_CT_ID_MUST_NOT_BE_ZERO = 5,
    TB_CT_ID_MUST_NOT_BE_INT_MAX = 6,
    TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 7,
    TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 8,
    TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 9,
    TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 10,
    TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 11,
    TB_CT_ACCOUNTS_MUST_BE_DIFFERENT = 12,
    TB_CT_PENDING_ID_MUST_BE_ZERO = 13,
    TB_CT_PENDING_ID_MUST_NOT_BE_ZERO = 14,
    TB_CT_PENDING_ID_MUST_NOT_BE_INT_MAX = 15,
    TB_CT_PENDING_ID_MUST_BE_DIFFERENT = 16,
    TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER = 17,
    TB_CT_DEPRECATED_18 = 18,
    TB_CT_LEDGER_MUST_NOT_BE_ZERO = 19,
    TB_CT_CODE_MUST_NOT_BE_ZERO = 20,
    TB_CT_DEBIT_ACCOUNT_NOT_FOUND = 21,
    TB_CT_CREDIT_ACCOUNT_NOT_FOUND = 22,
    TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER = 23,
    TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS = 24,
    TB_CT_PENDING_TRANSFER_NOT_FOUND = 25,
    TB_CT_PENDING_TRANSFER_NOT_PENDING = 26,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID = 27,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID = 28,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER = 29,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE = 30,
    TB_CT_EXCEEDS_PENDING_TRANSFER_AMOUNT = 31,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT = 32,
    TB_CT_PENDING_TRANSFER_ALREADY_POSTED = 33,
    TB_CT_PENDING_TRANSFER_ALREADY_VOIDED = 34,
    TB_CT_PENDING_TRANSFER_EXPIRED = 35,
    TB_CT_EXISTS_WITH_DIFFERENT_FLAGS = 36,
    TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID = 37,
    TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID = 38,
    TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT = 39,
    TB_CT_EXISTS_WITH_DIFFERENT_PENDING_ID = 40,
    TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 41,
    TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 42,
    TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 43,
    TB_CT_EXISTS_WITH_DIFFERENT_TIMEOUT = 44,
    TB_CT_EXISTS_WITH_DIFFERENT_CODE = 45,
    TB_CT_EXISTS = 46,
    TB_CT_OVERFLOWS_DEBITS_PENDING = 47,
    TB_CT_OVERFLOWS_CREDITS_PENDING = 48,
    TB_CT_OVERFLOWS_DEBITS_POSTED = 49,
    TB_CT_OVERFLOWS_CREDITS_POSTED = 50,
    TB_CT_OVERFLOWS_DEBITS = 51,
    TB_CT_OVERFLOWS_CREDITS = 52,
    TB_CT_OVERFLOWS_TIMEOUT = 53,
    TB_CT_EXCEEDS_CREDITS = 54,
    TB_CT_EXCEEDS_DEBITS = 55,
    TB_CT_IMPORTED_EVENT_EXPECTED = 56,
    TB_CT_IMPORTED_EVENT_NOT_EXPECTED = 57,
    TB_CT_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE = 58,
    TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_ADVANCE = 59,
    TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS = 60,
    TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_POSTDATE_DEBIT_ACCOUNT = 61,
    TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_POSTDATE_CREDIT_ACCOUNT = 62,
    TB_CT_IMPORTED_EVENT_TIMEOUT_MUST_BE_ZERO = 63,
    TB_CT_CLOSING_TRANSFER_MUST_BE_PENDING = 64,
    TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED = 65,
    TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED = 66,
    TB_CT_EXISTS_WITH_DIFFERENT_LEDGER = 67,
    TB_CT_ID_ALREADY_FAILED = 68,
};

/* src/lsm/timestamp_range.zig: timestamp_min = 1, timestamp_max = maxInt(u63). */
#define TB_TIMESTAMP_MIN 1ull
#define TB_TIMESTAMP_MAX 0x7FFFFFFFFFFFFFFFull
#define TB_NS_PER_S 1000000000ull

#if defined(__HIPCC__)
#define TB_INLINE __host__ __device__ static inline
#else
#define TB_INLINE static inline
#endif

/* CreateTransferStatus.transient(), src/tigerbeetle.zig:322-399. */
TB_INLINE int tb_transfer_status_transient(uint32_t s) {
    return s == TB_CT_DEBIT_ACCOUNT_NOT_FOUND || s == TB_CT_CREDIT_ACCOUNT_NOT_FOUND ||
           s == TB_CT_PENDING_TRANSFER_NOT_FOUND || s == TB_CT_EXCEEDS_CREDITS ||
           s == TB_CT_EXCEEDS_DEBITS || s == TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED ||
           s == TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED;
}

#ifdef __cplusplus
}  /* extern "C" */
static_assert(sizeof(tb_account_t) == 128, "Account must be 128 bytes");
static_assert(sizeof(tb_transfer_t) == 128, "Transfer must be 128 bytes");
static_assert(sizeof(tb_create_result_t) == 16, "Create*Result must be 16 bytes");
static_assert(offsetof(tb_account_t, user_data_64) == 96, "Account layout");
static_assert(offsetof(tb_account_t, ledger) == 112, "Account layout");
static_assert(offsetof(tb_account_t, code) == 116, "Account layout");
static_assert(offsetof(tb_account_t, flags) == 118, "Account layout");
static_assert(offsetof(tb_account_t, timestamp) == 120, "Account layout");
static_assert(offsetof(tb_transfer_t, user_data_64) == 96, "Transfer layout");
static_assert(offsetof(tb_transfer_t, timeout) == 108, "Transfer layout");
static_assert(offsetof(tb_transfer_t, ledger) == 112, "Transfer layout");
static_assert(offsetof(tb_transfer_t, code) == 116, "Transfer layout");
static_assert(offsetof(tb_transfer_t, flags) == 118, "Transfer layout");
static_assert(offsetof(tb_transfer_t, timestamp) == 120, "Transfer layout");
static_assert(sizeof(tb_account_event_t) == 256, "AccountEvent must be 256 bytes");
static_assert(offsetof(tb_account_event_t, timestamp) == 160, "AccountEvent layout");
static_assert(offsetof(tb_account_event_t, dr_account_flags) == 184, "AccountEvent layout");
static_assert(offsetof(tb_account_event_t, transfer_pending_id) == 192, "AccountEvent layout");
static_assert(offsetof(tb_account_event_t, ledger) == 240, "AccountEvent layout");
static_assert(offsetof(tb_account_event_t, transfer_pending_status) == 244, "AccountEvent layout");
static_assert(sizeof(tb_change_event_t) == 384, "ChangeEvent must be 384 bytes");
static_assert(offsetof(tb_change_event_t, ledger) == 84, "ChangeEvent layout");
static_assert(offsetof(tb_change_event_t, type) == 88, "ChangeEvent layout");
static_assert(offsetof(tb_change_event_t, debit_account_id) == 128, "ChangeEvent layout");
static_assert(offsetof(tb_change_event_t, credit_account_id) == 240, "ChangeEvent layout");
static_assert(offsetof(tb_change_event_t, timestamp) == 352, "ChangeEvent layout");
static_assert(sizeof(tb_change_events_filter_t) == 64, "ChangeEventsFilter must be 64 bytes");
static_assert(sizeof(tb_account_filter_t) == 128, "AccountFilter must be 128 bytes");
static_assert(offsetof(tb_account_filter_t, timestamp_min) == 104, "AccountFilter layout");
static_assert(sizeof(tb_query_filter_t) == 64, "QueryFilter must be 64 bytes");
static_assert(offsetof(tb_query_filter_t, timestamp_min) == 40, "QueryFilter layout");
static_assert(sizeof(tb_account_balance_t) == 128, "AccountBalance must be 128 bytes");
#else
_Static_assert(sizeof(tb_account_event_t) == 256, "AccountEvent must be 256 bytes");
_Static_assert(sizeof(tb_change_event_t) == 384, "ChangeEvent must be 384 bytes");
_Static_assert(sizeof(tb_change_events_filter_t) == 64, "ChangeEventsFilter must be 64 bytes");
_Static_assert(sizeof(tb_account_filter_t) == 128, "AccountFilter must be 128 bytes");
_Static_assert(offsetof(tb_account_filter_t, timestamp_min) == 104, "AccountFilter layout");
_Static_assert(sizeof(tb_query_filter_t) == 64, "QueryFilter must be 64 bytes");
_Static_assert(offsetof(tb_query_filter_t, timestamp_min) == 40, "QueryFilter layout");
_Static_assert(sizeof(tb_account_balance_t) == 128, "AccountBalance must be 128 bytes");
_Static_assert(sizeof(tb_account_t) == 128, "Account must be 128 bytes");
_Static_assert(sizeof(tb_transfer_t) == 128, "Transfer must be 128 bytes");
_Static_assert(sizeof(tb_create_result_t) == 16, "Create*Result must be 16 bytes");
_Static_assert(offsetof(tb_account_t, timestamp) == 120, "Account layout");
_Static_assert(offsetof(tb_transfer_t, timestamp) == 120, "Transfer layout");
#endif

#endif /* TB_TYPES_H */
