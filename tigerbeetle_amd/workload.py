"""Seeded synthetic workloads for the commit path (BASELINE.json configs).

All generators are numpy-vectorised and return records in the reference's extern layouts
(ACCOUNT_DTYPE / TRANSFER_DTYPE). Ids are sequential (``--id-order=sequential``,
src/testing/id.zig:29-31). Distributions follow src/tigerbeetle/benchmark_load.zig:941-1020:
uniform account choice with the credit index bumped on collision, ``code = rand(u16) +| 1``,
``amount = Exp(mean 10_000) +| 1``.
"""
import numpy as np

from .types import ACCOUNT_DTYPE, TRANSFER_DTYPE, AccountFlags, TransferFlags

U64 = np.uint64


def _u128_col(a, name, lo, hi=None):
    a[name][:, 0] = lo
    a[name][:, 1] = 0 if hi is None else hi


def accounts(n: int, seed: int = 42, id_offset: int = 0, ledger=2, code: int = 1,
             flags=None) -> np.ndarray:
    """`n` accounts with ids id_offset+1 .. id_offset+n (benchmark_load.zig:941-963)."""
    rng = np.random.default_rng(seed)
    a = np.zeros(n, dtype=ACCOUNT_DTYPE)
    _u128_col(a, "id", np.arange(id_offset + 1, id_offset + n + 1, dtype=U64))
    a["user_data_128"] = rng.integers(0, 2**63, size=(n, 2), dtype=np.int64).astype(U64)
    a["user_data_64"] = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(U64)
    a["user_data_32"] = rng.integers(0, 2**32, size=n, dtype=np.int64).astype(np.uint32)
    a["ledger"] = ledger
    a["code"] = code
    a["flags"] = int(AccountFlags.history) if flags is None else flags
    return a


def _codes(rng, n):
    r = rng.integers(0, 2**16, size=n, dtype=np.int64)
    return np.minimum(r + 1, 0xFFFF).astype(np.uint16)  # rand(u16) +| 1


def _amounts(rng, n, mean=10_000, amounts="exp"):
    """Exp(mean) +| 1 (benchmark_load.zig's), or with amounts="wide" log-uniform over
    [1, 2^63): most above 2^19, a ledger in cents moving up to ~$10^16 a transfer."""
    if amounts == "wide":
        e = np.floor(np.exp2(rng.uniform(0.0, 63.0, size=n)))
        return np.minimum(e, float(2**63 - 1024)).astype(U64)
    e = np.floor(rng.exponential(mean, size=n)).astype(np.int64)
    return (e + 1).astype(U64)  # Exp(mean) +| 1


def transfers_uniform(n: int, n_accounts: int, seed: int = 42, id_offset: int = 0,
                      account_id_offset: int = 0, ledger: int = 2,
                      amounts: str = "exp") -> np.ndarray:
    """Config 1/2: uniform debit/credit over the accounts, no pending (benchmark_load.zig:965)."""
    rng = np.random.default_rng(seed)
    t = np.zeros(n, dtype=TRANSFER_DTYPE)
    _u128_col(t, "id", np.arange(id_offset + 1, id_offset + n + 1, dtype=U64))
    dr = rng.integers(0, n_accounts, size=n, dtype=np.int64)
    cr = rng.integers(0, n_accounts, size=n, dtype=np.int64)
    cr = np.where(cr == dr, (cr + 1) % n_accounts, cr)
    _u128_col(t, "debit_account_id", (dr + 1 + account_id_offset).astype(U64))
    _u128_col(t, "credit_account_id", (cr + 1 + account_id_offset).astype(U64))
    t["user_data_128"] = rng.integers(0, 2**63, size=(n, 2), dtype=np.int64).astype(U64)
    t["user_data_64"] = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(U64)
    t["user_data_32"] = rng.integers(0, 2**32, size=n, dtype=np.int64).astype(np.uint32)
    t["ledger"] = ledger
    t["code"] = _codes(rng, n)
    _u128_col(t, "amount", _amounts(rng, n, amounts=amounts))
    return t


def zipf_indices(rng, n_items: int, theta: float, size: int) -> np.ndarray:
    """Zipfian ranks in [0, n_items) with P(i) ~ 1/(i+1)^theta."""
    w = 1.0 / np.power(np.arange(1, n_items + 1, dtype=np.float64), theta)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.searchsorted(cdf, rng.random(size), side="right").clip(0, n_items - 1)


def hot_limits_setup(n_accounts: int = 10_000, n_hot: int = 100, seed: int = 42,
                     funding: int = 2_000_000):
    """Config 3 accounts + funding transfers.

    Account 1 is an unlimited source; accounts 2..n_hot+1 are `hot` with
    debits_must_not_exceed_credits; the rest are cold. The funding transfers credit every hot
    account `funding` units from the source so that a fraction of hot debits later exceeds
    credits.
    """
    a = accounts(n_accounts, seed=seed)
    a["flags"][1:n_hot + 1] |= int(AccountFlags.debits_must_not_exceed_credits)
    f = np.zeros(n_hot, dtype=TRANSFER_DTYPE)
    return a, f, funding


def transfers_hot_limits(n: int, n_accounts: int = 10_000, n_hot: int = 100, seed: int = 42,
                         id_offset: int = 0, theta: float = 0.99, hot_debit_ratio: float = 0.9,
                         hot_credit_ratio: float = 0.1, amount_mean: int = 10_000,
                         amounts: str = "exp") -> np.ndarray:
    """Config 3: 90% of debits from Zipf-chosen hot (limited) accounts, ~10% of credits to hot."""
    rng = np.random.default_rng(seed)
    t = transfers_uniform(n, n_accounts, seed=seed + 1, id_offset=id_offset, amounts=amounts)
    cold_lo, cold_n = n_hot + 1, n_accounts - n_hot - 1  # cold indices [n_hot+1, n_accounts)
    hot = rng.random(n) < hot_debit_ratio
    dr = np.where(hot, 1 + zipf_indices(rng, n_hot, theta, n),
                  cold_lo + rng.integers(0, cold_n, size=n))
    to_hot = rng.random(n) < hot_credit_ratio
    cr = np.where(to_hot, 1 + rng.integers(0, n_hot, size=n),
                  cold_lo + rng.integers(0, cold_n, size=n))
    cr = np.where(cr == dr, np.where(cr + 1 < n_accounts, cr + 1, cold_lo), cr)
    _u128_col(t, "debit_account_id", (dr + 1).astype(U64))
    _u128_col(t, "credit_account_id", (cr + 1).astype(U64))
    _u128_col(t, "amount", _amounts(rng, n, amount_mean, amounts))
    return t


def funding_transfers(n_hot: int, amount, id_offset: int, source_index: int = 0):
    """One transfer per hot account from the unlimited source (account index 0 -> id 1);
    `amount` is one value for all or one per hot account."""
    t = np.zeros(n_hot, dtype=TRANSFER_DTYPE)
    _u128_col(t, "id", np.arange(id_offset + 1, id_offset + n_hot + 1, dtype=U64))
    _u128_col(t, "debit_account_id", np.full(n_hot, source_index + 1, dtype=U64))
    _u128_col(t, "credit_account_id", np.arange(2, n_hot + 2, dtype=U64))
    if isinstance(amount, (list, tuple)):  # u128 Python ints
        t["amount"][:, 0] = [a & 0xFFFFFFFFFFFFFFFF for a in amount]
        t["amount"][:, 1] = [a >> 64 for a in amount]
    else:
        _u128_col(t, "amount", np.broadcast_to(np.asarray(amount, dtype=U64), (n_hot,)).copy())
    t["ledger"] = 2
    t["code"] = 1
    return t


def hot_funding_amounts(t: np.ndarray, n_hot: int = 100, fraction: float = 0.8) -> np.ndarray:
    """Config 3 funding per hot account: `fraction` of what the stream `t` debits from it, less
    what the stream credits to it -- so that roughly the last (1 - fraction) of each hot
    account's debits find its credits exhausted (exceeds_credits)."""
    dr = t["debit_account_id"][:, 0].astype(np.int64) - 2   # hot accounts are ids 2..n_hot+1
    cr = t["credit_account_id"][:, 0].astype(np.int64) - 2
    amt = t["amount"][:, 0].astype(np.float64)
    hot_d, hot_c = (dr >= 0) & (dr < n_hot), (cr >= 0) & (cr < n_hot)
    debits = np.bincount(dr[hot_d], weights=amt[hot_d], minlength=n_hot)
    credits = np.bincount(cr[hot_c], weights=amt[hot_c], minlength=n_hot)
    f = np.maximum(fraction * debits - credits, 0)
    if f.max() >= 2.0**63:  # (wide amounts: u128 funding, as Python ints)
        return [int(x) for x in f]
    return f.astype(U64)


def transfers_two_phase(n: int, n_accounts: int, seed: int, id_offset: int,
                        prior_pending_ids: np.ndarray, pending_ratio=0.3, chain_ratio=0.3,
                        chain_len=8, fail_ratio=0.1, resubmit_ratio=0.01,
                        prior_ids: np.ndarray = None, prior_resolved_ids: np.ndarray = None,
                        n_limited: int = 0, amounts: str = "exp") -> np.ndarray:
    """Config 4: pending transfers with 1-5 s timeouts; posts (67%: half of them
    the full amount via maxInt, half a quarter of it) and voids (33%: 70% amount 0, 30% a nonzero
    amount, which fails with pending_transfer_has_different_amount when below the pending amount)
    of earlier pending transfers; 8-event linked chains on `chain_ratio` of the events, a
    `fail_ratio` of them with one injected failure at a random position -- a missing account, a
    ledger mismatch, `exceeds_credits` (a debit of one of the `n_limited` accounts 1..n_limited,
    which the caller creates with debits_must_not_exceed_credits, far beyond its credits; needs
    n_limited > 0) or a post of a pending transfer already posted or voided (`prior_resolved_ids`)
    -- and `resubmit_ratio` of ids resubmitted (exists / id_already_failed)."""
    rng = np.random.default_rng(seed)
    t = transfers_uniform(n, n_accounts, seed=seed, id_offset=id_offset, amounts=amounts)
    if n_limited:  # plain transfers never touch the limited accounts (their failures are injected)
        for col in ("debit_account_id", "credit_account_id"):
            low = t[col][:, 0] <= U64(n_limited)
            t[col][low, 0] = rng.integers(n_limited + 1, n_accounts + 1, size=int(low.sum()),
                                          dtype=np.int64).astype(U64)
        same = t["debit_account_id"][:, 0] == t["credit_account_id"][:, 0]
        t["credit_account_id"][same, 0] = np.where(
            t["credit_account_id"][same, 0] < U64(n_accounts), t["credit_account_id"][same, 0] + U64(1),
            U64(n_limited + 1))
    kind = rng.random(n)
    pend = kind < pending_ratio
    t["flags"][pend] |= int(TransferFlags.pending)
    t["timeout"][pend] = rng.integers(1, 6, size=int(pend.sum()), dtype=np.int64)
    if prior_pending_ids is not None and len(prior_pending_ids):
        resolve = (~pend) & (kind < pending_ratio + 0.3)
        idx = np.nonzero(resolve)[0]
        pick = prior_pending_ids[rng.integers(0, len(prior_pending_ids), size=len(idx))]
        post = rng.random(len(idx)) < 0.67
        t["flags"][idx] = np.where(post, int(TransferFlags.post_pending_transfer),
                                   int(TransferFlags.void_pending_transfer)).astype(np.uint16)
        t["pending_id"][idx, 0] = pick
        t["pending_id"][idx, 1] = 0
        # Post: amount maxInt half the time (post the full pending amount), else <= pending.
        # Void: amount 0 (the pending amount) 70% of the time, else a nonzero amount.
        full = rng.random(len(idx)) < 0.5
        void_amount = rng.random(len(idx)) < 0.3
        amt = t["amount"][idx, 0]
        t["amount"][idx, 0] = np.where(post & full, np.uint64(2**64 - 1),
                                       np.where(post | void_amount, amt // 4, 0))
        t["amount"][idx, 1] = np.where(post & full, np.uint64(2**64 - 1), 0)
        t["debit_account_id"][idx] = 0
        t["credit_account_id"][idx] = 0
        t["ledger"][idx] = 0
        t["code"][idx] = 0
        t["timeout"][idx] = 0
    # Linked chains of `chain_len` events, some with an injected failure.
    n_chains = int(n * chain_ratio / chain_len)
    starts = rng.choice(max(n - chain_len, 1), size=n_chains, replace=False) if n > chain_len else []
    kinds = ["missing", "ledger"] + (["exceeds_credits"] if n_limited else []) + \
            (["resolved"] if prior_resolved_ids is not None and len(prior_resolved_ids) else [])
    for s in sorted(starts):
        t["flags"][s:s + chain_len - 1] |= int(TransferFlags.linked)
        t["flags"][s + chain_len - 1] &= ~np.uint16(int(TransferFlags.linked))
        if rng.random() < fail_ratio:
            j = s + int(rng.integers(0, chain_len))
            what = kinds[int(rng.integers(0, len(kinds)))]
            if what == "missing":
                t["debit_account_id"][j] = [n_accounts + 1000, 0]
            elif what == "ledger":
                t["ledger"][j] = t["ledger"][j] + 1
                if (t["flags"][j] & (int(TransferFlags.post_pending_transfer) |
                                     int(TransferFlags.void_pending_transfer))):
                    t["ledger"][j] = 7  # pending_transfer_has_different_ledger
            elif what == "exceeds_credits":
                f = int(t["flags"][j]) & int(TransferFlags.linked)
                t["flags"][j] = f
                t["pending_id"][j] = 0
                t["timeout"][j] = 0
                t["code"][j] = 1
                t["ledger"][j] = 2
                t["debit_account_id"][j] = [1 + int(rng.integers(0, n_limited)), 0]
                t["credit_account_id"][j] = [n_limited + 1 + int(rng.integers(0, n_accounts - n_limited)), 0]
                t["amount"][j] = [2**40, 0]
            else:  # post of a pending transfer that was already posted or voided
                f = int(t["flags"][j]) & int(TransferFlags.linked)
                t["flags"][j] = f | int(TransferFlags.post_pending_transfer)
                t["pending_id"][j] = [int(prior_resolved_ids[rng.integers(0, len(prior_resolved_ids))]), 0]
                t["amount"][j] = [2**64 - 1, 2**64 - 1]
                t["debit_account_id"][j] = 0
                t["credit_account_id"][j] = 0
                t["ledger"][j] = 0
                t["code"][j] = 0
                t["timeout"][j] = 0
    # Resubmitted ids.
    if prior_ids is not None and len(prior_ids):
        m = int(n * resubmit_ratio)
        idx = rng.choice(n, size=m, replace=False)
        t["id"][idx, 0] = prior_ids[rng.integers(0, len(prior_ids), size=m)]
    return t


def fuzz_accounts(rng, n: int, id_space: int) -> np.ndarray:
    """Edge-biased create_accounts events (valid and invalid mixed)."""
    a = accounts(n, seed=int(rng.integers(0, 2**31)))
    a["id"][:, 0] = rng.integers(1, id_space + 1, size=n).astype(U64)
    a["ledger"] = rng.choice([1, 1, 1, 2, 0], size=n)
    a["code"] = rng.choice([1, 1, 1, 2, 0], size=n)
    fl = np.zeros(n, dtype=np.int64)
    for bit, p in ((0, 0.15), (1, 0.25), (2, 0.15), (3, 0.3), (5, 0.05)):
        fl |= (rng.random(n) < p).astype(np.int64) << bit
    a["flags"] = fl.astype(np.uint16)
    a["reserved"] = (rng.random(n) < 0.02).astype(np.uint32)
    a["timestamp"] = (rng.random(n) < 0.02).astype(U64)
    a["debits_posted"][:, 0] = (rng.random(n) < 0.02).astype(U64)
    a["id"][rng.random(n) < 0.01] = 0
    return a


def fuzz_transfers(rng, n: int, id_space: int, n_accounts: int, pending_ids=None) -> np.ndarray:
    """Edge-biased create_transfers events covering every status path."""
    t = transfers_uniform(n, n_accounts, seed=int(rng.integers(0, 2**31)))
    t["ledger"] = rng.choice([1, 1, 1, 1, 2, 0], size=n)
    t["id"][:, 0] = rng.integers(1, id_space + 1, size=n).astype(U64)
    dr = rng.integers(1, n_accounts + 3, size=n)
    cr = rng.integers(1, n_accounts + 3, size=n)
    t["debit_account_id"][:, 0] = dr.astype(U64)
    t["credit_account_id"][:, 0] = cr.astype(U64)
    small = rng.random(n) < 0.5
    t["amount"][:, 0] = np.where(small, rng.integers(0, 50, size=n), t["amount"][:, 0]).astype(U64)
    big = rng.random(n) < 0.03
    t["amount"][big, 0] = np.uint64(2**64 - 1)
    t["amount"][big, 1] = np.uint64(2**64 - 1)
    fl = np.zeros(n, dtype=np.int64)
    for bit, p in ((0, 0.2), (1, 0.3), (2, 0.12), (3, 0.08), (4, 0.08), (5, 0.08), (6, 0.03),
                   (7, 0.03)):
        fl |= (rng.random(n) < p).astype(np.int64) << bit
    fl |= (rng.random(n) < 0.01).astype(np.int64) << 10  # padding
    t["flags"] = fl.astype(np.uint16)
    pend = (fl & int(TransferFlags.pending)) != 0
    t["timeout"] = np.where(pend & (rng.random(n) < 0.5), rng.integers(1, 4, size=n), 0)
    t["timeout"][rng.random(n) < 0.02] = 7
    pv = (fl & (int(TransferFlags.post_pending_transfer) |
                int(TransferFlags.void_pending_transfer))) != 0
    if pending_ids is not None and len(pending_ids):
        pick = pending_ids[rng.integers(0, len(pending_ids), size=n)]
        t["pending_id"][:, 0] = np.where(pv, pick, 0).astype(U64)
    else:
        t["pending_id"][:, 0] = np.where(pv, rng.integers(1, id_space + 1, size=n), 0).astype(U64)
    zero_acc = pv & (rng.random(n) < 0.7)
    t["debit_account_id"][zero_acc] = 0
    t["credit_account_id"][zero_acc] = 0
    t["ledger"][zero_acc & (rng.random(n) < 0.7)] = 0
    t["code"][pv & (rng.random(n) < 0.5)] = 0
    t["code"][rng.random(n) < 0.01] = 0
    t["timestamp"] = (rng.random(n) < 0.01).astype(U64)
    t["id"][rng.random(n) < 0.005] = 0
    return t


# ---- config 5: many accounts over 64 ledgers, sharded by ledger ----------

LEDGERS_CONFIG5 = 64


def config5_ledgers(rank: int, world: int):
    """The rank's contiguous ledger range: (first ledger offset, ledgers per shard)."""
    if LEDGERS_CONFIG5 % world:
        raise ValueError(f"{LEDGERS_CONFIG5} ledgers do not split over {world} shards")
    per = LEDGERS_CONFIG5 // world
    return rank * per, per


def config5_global_index(j: np.ndarray, rank: int, world: int) -> np.ndarray:
    """Global account index k of the rank's local account j: account k lives on ledger
    1 + (k mod 64); the rank holds the accounts of its ledgers, interleaved by ledger."""
    first, per = config5_ledgers(rank, world)
    j = np.asarray(j, dtype=np.int64)
    return (j // per) * LEDGERS_CONFIG5 + first + (j % per)


def accounts_config5(j: np.ndarray, rank: int, world: int) -> np.ndarray:
    """The rank's local accounts `j` (id = global index + 1, ledger 1 + (k mod 64), code 1,
    history; user data a fixed function of the id, so any subset is reproducible)."""
    k = config5_global_index(j, rank, world)
    n = len(k)
    # Written through a (n, 16) u64 view of the records (word w = bytes 8w..8w+7).
    w = np.zeros((n, 16), dtype=U64)
    ids = (k + 1).astype(U64)
    w[:, 0] = ids                                              # id (lo)
    with np.errstate(over="ignore"):
        w[:, 10] = ids * U64(0x9E3779B97F4A7C15)               # user_data_128
        w[:, 11] = ids * U64(0xC2B2AE3D27D4EB4F)
        w[:, 12] = ids * U64(0x165667B19E3779F9)               # user_data_64
    w[:, 13] = ids & U64(0xFFFFFFFF)                           # user_data_32, reserved 0
    # ledger (u32) | code (u16) << 32 | flags (u16) << 48
    w[:, 14] = ((1 + (k % LEDGERS_CONFIG5)).astype(U64) | (U64(1) << U64(32)) |
                (U64(int(AccountFlags.history)) << U64(48)))
    return w.view(ACCOUNT_DTYPE).reshape(n)


def transfers_config5(n: int, accounts_per_shard: int, rank: int, world: int, seed: int = 42,
                      id_offset: int = 0):
    """`n` transfers of the rank's shard: a ledger uniform over the shard's ledgers, then debit and
    credit uniform within it (credit bumped on collision). Returns (transfers, dr_local,
    cr_local), the local account indices for validation."""
    first, per = config5_ledgers(rank, world)
    groups = accounts_per_shard // per
    if groups < 2:
        raise ValueError("config 5 needs at least two accounts per ledger")
    rng = np.random.default_rng(seed + 7919 * rank)
    lo = rng.integers(0, per, size=n, dtype=np.int64)
    gd = rng.integers(0, groups, size=n, dtype=np.int64)
    gc = rng.integers(0, groups, size=n, dtype=np.int64)
    gc = np.where(gc == gd, (gc + 1) % groups, gc)
    dr_local, cr_local = gd * per + lo, gc * per + lo
    t = np.zeros(n, dtype=TRANSFER_DTYPE)
    _u128_col(t, "id", np.arange(id_offset + 1, id_offset + n + 1, dtype=U64))
    _u128_col(t, "debit_account_id", (config5_global_index(dr_local, rank, world) + 1).astype(U64))
    _u128_col(t, "credit_account_id", (config5_global_index(cr_local, rank, world) + 1).astype(U64))
    t["user_data_64"] = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(U64)
    t["ledger"] = (1 + first + lo).astype(np.uint32)
    t["code"] = _codes(rng, n)
    _u128_col(t, "amount", _amounts(rng, n))
    return t, dr_local, cr_local


# ---- the sharded group's workloads (bench.py group lines, tests/test_routed.py) -----------------

HAZARD_KINDS = ("debit_not_found", "cross_ledger", "id_zero", "reserved_flag", "repeat_exists",
                "pending_not_found", "credit_not_found")


def group_accounts(ledgers: int, per_ledger: int, seed: int = 42) -> np.ndarray:
    """`per_ledger` accounts on each of ledgers 2 .. ledgers + 1 (ids (ledger - 2) * per_ledger + 1
    ..): the group's shards by ledger (ledger range option `ledgers + 1`)."""
    return np.concatenate([accounts(per_ledger, seed=seed + i, id_offset=i * per_ledger,
                                    ledger=2 + i) for i in range(ledgers)])


def mixed_ledger_transfers(n: int, ledgers: int, per_ledger: int, seed: int = 42,
                           id_offset: int = 0):
    """One client call of `n` transfers whose ledger is uniform per event over ledgers 2 ..
    ledgers + 1, debit / credit uniform within it (benchmark_load.zig's distributions), ids
    id_offset + 1 ..; returns (transfers, ledger index per event)."""
    t = transfers_uniform(n, per_ledger, seed=seed, id_offset=id_offset)
    lg = np.random.default_rng(seed + 1).integers(0, ledgers, size=n).astype(U64)
    t["debit_account_id"][:, 0] += lg * U64(per_ledger)
    t["credit_account_id"][:, 0] += lg * U64(per_ledger)
    t["ledger"] = (2 + lg).astype(np.uint32)
    return t, lg


def hazard_transfers(n: int, ledgers: int, per_ledger: int, rate: float, seed: int = 42,
                     id_offset: int = 0):
    """mixed_ledger_transfers with a fraction `rate` of injected failures whose statuses follow
    from the events alone (config 4's failure kinds across ledgers; src/state_machine.zig
    :3729-3798, :4053-4100): an unknown debit / credit account, a credit account on another
    ledger (another shard), id 0, a reserved flag, a post of a pending transfer found nowhere, and
    an exact repeat of an earlier transfer of the call (`exists`). Returns (transfers, kinds: -1 or
    the HAZARD_KINDS index per event, the repeated event's index per event or -1)."""
    if ledgers < 2:
        raise ValueError("hazard_transfers needs two ledgers at least (cross-ledger transfers)")
    t, lg = mixed_ledger_transfers(n, ledgers, per_ledger, seed=seed, id_offset=id_offset)
    rng = np.random.default_rng(seed + 2)
    m = max(1, int(n * rate))
    pos = np.sort(rng.choice(np.arange(n // 2, n), size=m, replace=False))
    kinds = np.full(n, -1, dtype=np.int64)
    src = np.full(n, -1, dtype=np.int64)
    unknown = U64(1 << 40)
    for j, k in enumerate(pos.tolist()):
        kind = j % len(HAZARD_KINDS)
        kinds[k] = kind
        name = HAZARD_KINDS[kind]
        if name == "debit_not_found":
            t["debit_account_id"][k, 0] = unknown + U64(k)
        elif name == "credit_not_found":
            t["credit_account_id"][k, 0] = unknown + U64(k)
        elif name == "cross_ledger":
            other = (int(lg[k]) + 1) % ledgers
            t["credit_account_id"][k, 0] = U64(other * per_ledger + 1 + k % per_ledger)
        elif name == "id_zero":
            t["id"][k] = 0
        elif name == "reserved_flag":
            t["flags"][k] = 1 << 12
        elif name == "pending_not_found":
            t["flags"][k] = 4  # post_pending_transfer
            t["pending_id"][k, 0] = unknown + U64(k)
        elif name == "repeat_exists":
            s = int(rng.integers(0, n // 2))  # (the first half holds no injected event)
            t[k] = t[s]
            src[k] = s
    return t, kinds, src


def hazard_expected(t: np.ndarray, kinds: np.ndarray, src: np.ndarray, stamps: np.ndarray,
                    ledgers: int):
    """The reference's results for hazard_transfers (closed form; every other event is created,
    and no event's outcome depends on order) -- (status, timestamp) per event -- and the created
    events' mask."""
    from .types import CreateTransferStatus as S
    status = np.full(len(t), STATUS_CREATED_U32, dtype=np.uint32)
    ts = stamps.astype(U64).copy()
    want = {
        "debit_not_found": S.debit_account_not_found,
        "credit_not_found": S.credit_account_not_found,
        "cross_ledger": S.accounts_must_have_the_same_ledger,
        "id_zero": S.id_must_not_be_zero,
        "reserved_flag": S.reserved_flag,
        "pending_not_found": S.pending_transfer_not_found,
    }
    for kind, name in enumerate(HAZARD_KINDS):
        sel = kinds == kind
        if name == "repeat_exists":
            status[sel] = int(S.exists)
            ts[sel] = stamps[src[sel]]
        else:
            status[sel] = int(want[name])
    return status, ts, status == STATUS_CREATED_U32


STATUS_CREATED_U32 = 0xFFFFFFFF
