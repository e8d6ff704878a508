/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, called by, or shipped
 * with the product (libhftlob.so).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load liboracle.so, as the checker / CPU baseline.
 *
 * Plain-C, plain-loop restatement of the reference hot path of
 * biiiipy/JaxMARL-HFT (pure Python/JAX; nothing native to compile):
 *   order book      gymnax_exchange/jaxob/JaxOrderBookArrays.py
 *   MARL step/reset gymnax_exchange/jaxen/marl_env.py
 *   agents          gymnax_exchange/jaxen/mm_env.py, exec_env.py
 *   data windows    gymnax_exchange/jaxen/base_env.py
 *   JAX PRNG        jax.random threefry2x32 / split / randint / permutation
 *                   (third-party, version unpinned in requirements.txt:2;
 *                   restated from its published algorithm)
 * Each function cites the reference lines it follows.
 *
 * PARITY STATUS: the reference cannot run here (no jax) and ships no tests or
 * golden outputs, so this restatement is pinned only by (1) Random123
 * threefry2x32-20 known-answer vectors, (2) hand-derived micro-scenarios in
 * tests/golden, (3) agreement with the independent numpy restatement
 * oracle/ref_py.py.  Reference-generated vectors: none ("parity unpinned"
 * against the reference's own outputs).
 *
 * Float arithmetic is float32, op for op as XLA would evaluate the jnp
 * expressions (int32 operands promoted to f32, weak-typed Python constants
 * staying f32).  Float sums use the canonical "wave order" (fold element
 * l+64 into l, then xor-butterfly 1, 2, .., 32) so this checker matches the HIP path
 * bit for bit; the reference's own XLA order is unknowable, hence
 * the 1e-5 tolerance in the tests against the reference-order numpy oracle.
 * Build: cc -O2 -fopenmp -ffp-contract=off (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/hftlob.h"

typedef int32_t i32;
typedef uint32_t u32;

/* ------------------------------------------------------------------ ints */
static inline i32 wadd(i32 a, i32 b) { return (i32)((u32)a + (u32)b); }
static inline i32 wsub(i32 a, i32 b) { return (i32)((u32)a - (u32)b); }
static inline i32 wmul(i32 a, i32 b) { return (i32)((u32)a * (u32)b); }
static inline i32 imax(i32 a, i32 b) { return a > b ? a : b; }
static inline i32 imin(i32 a, i32 b) { return a < b ? a : b; }
static inline i32 iabs(i32 a) { return a < 0 ? wsub(0, a) : a; }
static inline i32 isign(i32 a) { return (a > 0) - (a < 0); }
/* jnp.floor_divide on int32 */
static inline i32 ifloordiv(i32 a, i32 b) {
    i32 q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
    return q;
}
/* jnp.floor_divide on float32: jax _float_divmod + round-half-away */
static inline float ffloordiv(float x, float y) {
    float mod = fmodf(x, y);
    float div = (x - mod) / y;
    int ind = (mod != 0.0f) && ((y > 0) - (y < 0)) != ((mod > 0) - (mod < 0));
    if (ind) div = div - 1.0f;
    return roundf(div);
}
static inline float i2f(i32 a) { return (float)a; }
static inline i32 f2i(float f) { return (i32)f; } /* XLA convert: truncation */

/* XLA f32 -> s32 convert (saturating; NaN -> 0) */
static i32 f2i_sat(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (i32)f;
}
/* jnp table[idx] on a traced index: negative indices wrap once, then clamp */
static int gather_idx(i32 a, int n) {
    i32 i = a < 0 ? a + n : a;
    return i < 0 ? 0 : (i >= n ? n - 1 : i);
}

static inline float bitf(i32 w) { float f; memcpy(&f, &w, 4); return f; }
static inline i32 fbit(float f) { i32 w; memcpy(&w, &f, 4); return w; }

/* canonical wave-order float sum: lane l folds x[l], x[l+64], x[l+128], ...
 * in that order, then an xor-butterfly over the 64 lanes (k = 1, 2, .. 32;
 * the HIP kernel's DPP reduction gives exactly this tree at lane 63) */
static float wsum(const float* x, int n) {
    float v[64];
    for (int l = 0; l < 64; ++l) {
        float a = l < n ? x[l] : 0.0f;
        for (int j = l + 64; j < n; j += 64) a = a + x[j];
        v[l] = a;
    }
    for (int k = 1; k <= 32; k <<= 1) {  /* xor butterfly 1, 2, 4, 8, 16, 32 */
        float t[64];
        for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ k];
        memcpy(v, t, sizeof v);
    }
    return v[63];
}

/* ================================================================= PRNG */
static inline u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }

void oracle_threefry2x32(u32 k0, u32 k1, u32 x0, u32 x1, u32* o0, u32* o1) {
    static const int R[8] = {13, 15, 26, 6, 17, 29, 16, 24};
    u32 ks[3] = {k0, k1, k0 ^ k1 ^ 0x1BD11BDAu};
    x0 += ks[0];
    x1 += ks[1];
    for (int i = 1; i <= 5; ++i) {
        const int* r = (i & 1) ? R : R + 4;
        for (int j = 0; j < 4; ++j) {
            x0 += x1;
            x1 = rotl32(x1, r[j]);
            x1 ^= x0;
        }
        x0 += ks[i % 3];
        x1 += ks[(i + 1) % 3] + (u32)i;
    }
    *o0 = x0;
    *o1 = x1;
}

/* jax.random.split(key, n)[j] */
void oracle_split(const u32* key, int n, int j, int part, u32* out) {
    if (part) {
        oracle_threefry2x32(key[0], key[1], 0u, (u32)j, &out[0], &out[1]);
        return;
    }
    /* legacy: counts iota(2n) split in halves, outputs concatenated, (n,2) */
    for (int w = 0; w < 2; ++w) {
        int m = 2 * j + w; /* flat output index */
        u32 y0, y1;
        if (m < n) {
            oracle_threefry2x32(key[0], key[1], (u32)m, (u32)(n + m), &y0, &y1);
            out[w] = y0;
        } else {
            oracle_threefry2x32(key[0], key[1], (u32)(m - n), (u32)m, &y0, &y1);
            out[w] = y1;
        }
    }
}

/* jax random_bits(key, 32, (n,)) element i */
static u32 random_bits_i(const u32* key, int n, int i, int part) {
    u32 y0, y1;
    if (part) {
        oracle_threefry2x32(key[0], key[1], 0u, (u32)i, &y0, &y1);
        return y0 ^ y1;
    }
    int half = (n + 1) / 2;
    if (i < half) {
        u32 x1 = (i + half < n) ? (u32)(i + half) : 0u;
        oracle_threefry2x32(key[0], key[1], (u32)i, x1, &y0, &y1);
        return y0;
    }
    u32 x1 = (i < n) ? (u32)i : 0u;
    oracle_threefry2x32(key[0], key[1], (u32)(i - half), x1, &y0, &y1);
    return y1;
}

/* jax.random.randint(key, (n,), lo, hi)[j] for int32 (jax/_src/random.py _randint: two
 * random_bits draws of the shape from split(key), folded modulo the span) */
static i32 randint_shaped(const u32* key, int n, int j, i32 lo, i32 hi, int part) {
    u32 k1[2], k2[2];
    oracle_split(key, 2, 0, part, k1);
    oracle_split(key, 2, 1, part, k2);
    u32 hb = random_bits_i(k1, n, j, part), lb = random_bits_i(k2, n, j, part);
    u32 span = (hi <= lo) ? 1u : (u32)hi - (u32)lo;
    u32 mult = 65536u % span;
    mult = (mult * mult) % span;
    u32 off = ((hb % span) * mult + (lb % span)) % span;
    return (i32)((u32)lo + off);
}

/* jax.random.randint(key, (), lo, hi) for int32 */
i32 oracle_randint(const u32* key, i32 lo, i32 hi, int part) { return randint_shaped(key, 1, 0, lo, hi, part); }

/* jax.random.permutation(key, arange(n)): perm[j] = source row of output j */
void oracle_permutation(const u32* key, int n, int part, int* perm) {
    for (int i = 0; i < n; ++i) perm[i] = i;
    if (n < 2) return; /* num_rounds = ceil(3 ln n / ln(2^32-1)) = 0 for n = 1 */
    u32 sub[2], bits[HFTLOB_MAX_MSGS];
    oracle_split(key, 2, 1, part, sub);
    for (int i = 0; i < n; ++i) bits[i] = random_bits_i(sub, n, i, part);
    for (int i = 1; i < n; ++i) { /* stable insertion sort by bits */
        u32 b = bits[i];
        int p = perm[i], j = i - 1;
        while (j >= 0 && bits[j] > b) {
            bits[j + 1] = bits[j];
            perm[j + 1] = perm[j];
            --j;
        }
        bits[j + 1] = b;
        perm[j + 1] = p;
    }
}

/* ========================================================= order book (L1) */
#ifdef ORACLE_STATS /* message-mix statistics (tools/msg_mix.py; single-threaded builds only) */
long long oracle_stats[32];
#define STAT(i) (oracle_stats[i]++)
/* per-message class trace (tools/msg_runs.py): 0 doNothing, 1 add behind / at the best, 2 add
 * improving the best, 3 crossing add, 4 add into a full side, 5 cancel of quantity 0, 6 cancel
 * found by id, 7 cancel found by the init-id fallback, 8 cancel of no row into an empty last
 * slot, 9 cancel of no row into an occupied last slot, 10 as 8 but an init-id row at the price
 * holds less than the cancel's quantity */
signed char oracle_trace[1 << 24];
long long oracle_trace_n;
#else
#define STAT(i) ((void)0)
#endif
typedef struct {
    i32 side, type, price, qty, oid, tid, t, tns;
} Msg;

/* _removeZeroNegQuant — JaxOrderBookArrays.py:85-90 */
static void remove_zero_neg(i32* s, int nO) {
    for (int i = 0; i < nO; ++i)
        if (s[i * 6 + 1] <= 0)
            for (int f = 0; f < 6; ++f) s[i * 6 + f] = -1;
}

/* add_order — :62-83: first row containing ANY -1 (row-major), -1 -> last */
static void add_order(i32* s, int nO, const Msg* m) {
    int idx = nO - 1;
    for (int i = 0; i < nO * 6; ++i)
        if (s[i] == -1) { idx = i / 6; break; }
    i32* r = s + idx * 6;
    r[0] = m->price; r[1] = imax(0, m->qty); r[2] = m->oid;
    r[3] = m->tid;   r[4] = m->t;            r[5] = m->tns;
    remove_zero_neg(s, nO);
}

/* get_random_id_match (large = 0) / get_random_large_id_match (large = 1) —
 * :141-164.  key <- split(key, 2)[0]; order_ids = where(price match [& qty >=
 * msg qty], oid, 0); chosen = jax.random.choice(key, order_ids,
 * p=|sign(order_ids)|), which for p given and shape () is
 *   p_cuml = cumsum(p) (float32); r = p_cuml[-1] * (1 - uniform(key));
 *   ind = searchsorted(p_cuml, r, side='left'); chosen = order_ids[ind]
 * (jax/_src/random.py choice; uniform = bits >> 9 | 1.0f, minus 1).  Then idx =
 * first row with oid == chosen, or -1. */
static int random_id_match(const hftlob_lob_cfg* c, u32* key, const i32* s, const Msg* m, int large) {
    int nO = c->n_orders, part = c->prng_partitionable;
    u32 k[2];
    oracle_split(key, 2, 0, part, k);
    key[0] = k[0];
    key[1] = k[1];
    i32 ids[HFTLOB_MAX_SLOTS];
    float cum[HFTLOB_MAX_SLOTS], acc = 0.0f;
    for (int i = 0; i < nO; ++i) {
        const i32* r = s + i * 6;
        int pm = r[0] == m->price && (large || r[1] >= m->qty);
        ids[i] = pm ? r[2] : 0;
        acc += (float)iabs(isign(ids[i]));
        cum[i] = acc;
    }
    u32 bits = random_bits_i(key, 1, 0, part), fb = (bits >> 9) | 0x3f800000u;
    float u;
    memcpy(&u, &fb, 4);
    u -= 1.0f;
    float r = cum[nO - 1] * (1.0f - u);
    int ind = 0;
    while (ind < nO && cum[ind] < r) ++ind;  /* searchsorted, side='left' */
    if (ind >= nO) ind = nO - 1;             /* unreachable: r <= cum[-1] */
    i32 chosen = ids[ind];
    for (int i = 0; i < nO; ++i)
        if (s[i * 6 + 2] == chosen) return i;
    return -1;
}

/* cancel_order + get_init_id_match — :93-139; cancel_mode 2/3 fall back to
 * the random matches (:130-136,149-154) drawing from `key` (the scan key of
 * this message, split(key, M)[k], :753,784,816) */
static void cancel_order(const hftlob_lob_cfg* c, i32* s, const Msg* m, const u32* msg_key) {
    int nO = c->n_orders, idx = -1;
    for (int i = 0; i < nO; ++i)
        if (s[i * 6 + 2] == m->oid) { idx = i; break; }
#ifdef ORACLE_STATS
    STAT(10);
    if (m->qty == 0) STAT(11);
    else if (idx >= 0) STAT(12);
#endif
    if (idx == -1) { /* get_init_id_match (called for every cancel mode) */
        i32 lo = wsub(c->init_id, wmul(c->book_depth, 2));
        for (int i = 0; i < nO; ++i) {
            const i32* r = s + i * 6;
            if (r[0] == m->price && r[2] <= c->init_id && r[2] >= lo && r[1] >= m->qty) { idx = i; break; }
        }
        if (idx == -1 && c->cancel_mode >= 2) {
            u32 k[2] = {msg_key[0], msg_key[1]};
            idx = random_id_match(c, k, s, m, 0);
            if (idx == -1 && c->cancel_mode == 3) idx = random_id_match(c, k, s, m, 1);
        }
    }
#ifdef ORACLE_STATS
    if (m->qty != 0 && idx >= 0 && s[idx * 6 + 2] != m->oid) STAT(21);   /* init-id fallback found */
    if (m->qty != 0 && idx == -1) { STAT(22); if (s[(nO - 1) * 6] == -1) STAT(23); }
#endif
    if (idx == -1) idx = nO - 1; /* negative index wraps to the last slot */
#ifdef ORACLE_STATS
    if (m->qty != 0) {
        if (s[idx * 6 + 1] - m->qty <= 0) STAT(13);          /* row removed */
        int bid = m->side == 1;
        i32 best = bid ? -1 : c->maxint;
        for (int i = 0; i < nO; ++i) {
            i32 p = s[i * 6];
            if (bid) best = imax(best, p); else if (p != -1) best = imin(best, p);
        }
        if (s[idx * 6] == best) STAT(14);                      /* at the best price */
    }
#endif
    s[idx * 6 + 1] = wsub(s[idx * 6 + 1], m->qty);
    remove_zero_neg(s, nO);
}

/* _get_top_bid_order_idx — :241-252 */
static int top_bid_idx(const i32* s, int nO, i32 maxint) {
    i32 mp = s[0];
    for (int i = 1; i < nO; ++i) mp = imax(mp, s[i * 6]);
    i32 mts = maxint;
    for (int i = 0; i < nO; ++i) mts = imin(mts, s[i * 6] == mp ? s[i * 6 + 4] : maxint);
    i32 mtn = maxint;
    for (int i = 0; i < nO; ++i) {
        i32 ts = s[i * 6] == mp ? s[i * 6 + 4] : maxint;
        mtn = imin(mtn, ts == mts ? s[i * 6 + 5] : maxint);
    }
    for (int i = 0; i < nO; ++i) {
        i32 ts = s[i * 6] == mp ? s[i * 6 + 4] : maxint;
        if ((ts == mts ? s[i * 6 + 5] : maxint) == mtn) return i;
    }
    return nO - 1; /* unreachable */
}

/* _get_top_ask_order_idx — :255-268 (empty slots' -1 price -> maxint) */
static int top_ask_idx(const i32* s, int nO, i32 maxint) {
    i32 mp = maxint;
    for (int i = 0; i < nO; ++i) mp = imin(mp, s[i * 6] == -1 ? maxint : s[i * 6]);
    i32 mts = maxint;
    for (int i = 0; i < nO; ++i) mts = imin(mts, s[i * 6] == mp ? s[i * 6 + 4] : maxint);
    i32 mtn = maxint;
    for (int i = 0; i < nO; ++i) {
        i32 ts = s[i * 6] == mp ? s[i * 6 + 4] : maxint;
        mtn = imin(mtn, ts == mts ? s[i * 6 + 5] : maxint);
    }
    for (int i = 0; i < nO; ++i) {
        i32 ts = s[i * 6] == mp ? s[i * 6 + 4] : maxint;
        if ((ts == mts ? s[i * 6 + 5] : maxint) == mtn) return i;
    }
    return nO - 1;
}

/* match_order — :172-220; trade row at first row whose col 4 == -1 */
static i32 match_order(i32* s, int nO, int top, i32 qtm, const Msg* m, i32* trades, int nT) {
    i32* r = s + top * 6;
    i32 newq = imax(0, wsub(r[1], qtm));
    i32 rem = wsub(qtm, r[1]);
#ifdef ORACLE_STATS
    if (newq <= 0) STAT(24);
#endif
    int e = nT - 1;
    for (int i = 0; i < nT; ++i)
        if (trades[i * 8 + 4] == -1) { e = i; break; }
    i32* t = trades + e * 8;
    t[0] = r[0]; t[1] = wmul(wsub(0, m->side), wsub(r[1], newq)); t[2] = r[2];
    t[3] = m->oid; t[4] = m->t; t[5] = m->tns; t[6] = r[3]; t[7] = m->tid;
    r[1] = newq;
    remove_zero_neg(s, nO);
    return rem;
}

/* _match_against_bid_orders / _match_against_ask_orders — :284-331 */
static i32 match_against(const hftlob_lob_cfg* c, i32* s, int bid_side, i32 qtm, i32 price,
                         const Msg* m, i32* trades) {
    int nO = c->n_orders;
    for (;;) {
        int top = bid_side ? top_bid_idx(s, nO, c->maxint) : top_ask_idx(s, nO, c->maxint);
        i32 tp = s[top * 6];
        int go = bid_side ? (tp >= price) : (tp <= price);
        if (!(go && qtm > 0 && tp != -1)) return qtm;
        STAT(20);
        qtm = match_order(s, nO, top, qtm, m, trades, c->n_trades);
    }
}

/* bid_lim — :357-420 (incoming buy) */
static void bid_lim(const hftlob_lob_cfg* c, Msg m, i32* asks, i32* bids, i32* trades) {
    int nO = c->n_orders;
    i32 rem = match_against(c, asks, 0, m.qty, m.price, &m, trades);
    if (c->type_4_interpretation == 2) m.price = c->maxint; /* after matching (sic) */
    m.qty = rem;
    if (c->check_book_fill) {
        int full = 1;
        i32 worst = bids[0];
        for (int i = 0; i < nO; ++i) { full &= bids[i * 6] >= 0; worst = imin(worst, bids[i * 6]); }
#ifdef ORACLE_STATS
        if (full) STAT(25);
#endif
        if (full)
            for (int i = 0; i < nO; ++i)
                if (bids[i * 6] == worst) for (int f = 0; f < 6; ++f) bids[i * 6 + f] = -1;
    }
    int discard = (c->type_4_interpretation == 0 || c->type_4_interpretation == 2) && m.type == 4;
    if (!discard) add_order(bids, nO, &m);
}

/* ask_lim — :446-508 (incoming sell) */
static void ask_lim(const hftlob_lob_cfg* c, Msg m, i32* asks, i32* bids, i32* trades) {
    int nO = c->n_orders;
    if (c->type_4_interpretation == 2) m.price = 0;
    i32 rem = match_against(c, bids, 1, m.qty, m.price, &m, trades);
    m.qty = rem;
    if (c->check_book_fill) {
        int full = 1;
        i32 worst = asks[0];
        for (int i = 0; i < nO; ++i) { full &= asks[i * 6] >= 0; worst = imax(worst, asks[i * 6]); }
#ifdef ORACLE_STATS
        if (full) STAT(25);
#endif
        if (full)
            for (int i = 0; i < nO; ++i)
                if (asks[i * 6] == worst) for (int f = 0; f < 6; ++f) asks[i * 6 + f] = -1;
    }
    int discard = (c->type_4_interpretation == 0 || c->type_4_interpretation == 2) && m.type == 4;
    if (!discard) add_order(asks, nO, &m);
}

/* get_best_bid_and_ask_inclQuants — :932-984 */
static void best_quotes(const hftlob_lob_cfg* c, const i32* asks, const i32* bids, i32* ba, i32* bb) {
    int nO = c->n_orders;
    i32 mn = c->maxint, mx = bids[0];
    for (int i = 0; i < nO; ++i) {
        mn = imin(mn, asks[i * 6] == -1 ? c->maxint : asks[i * 6]);
        mx = imax(mx, bids[i * 6]);
    }
    i32 pa = mn == c->maxint ? -1 : mn, qa = 0, qb = 0;
    for (int i = 0; i < nO; ++i) {
        if (asks[i * 6] == pa) qa = wadd(qa, asks[i * 6 + 1]);
        if (bids[i * 6] == mx) qb = wadd(qb, bids[i * 6 + 1]);
    }
    ba[0] = pa; ba[1] = qa; bb[0] = mx; bb[1] = qb;
}

/* cond_type_side_save_bidask — :687-732 (GENERAL_EXCHANGE mode) */
/* scan_key / n_msg / k: the scan's key and this message's position (the key
 * is split(scan_key, n_msg)[k]; only drawn from under cancel_mode 2/3) */
static void process_msg(const hftlob_lob_cfg* c, const i32* d, i32* asks, i32* bids, i32* trades,
                        const u32* scan_key, int n_msg, int k) {
    u32 mk[2] = {0u, 0u};
    if (c->cancel_mode >= 2) oracle_split(scan_key, n_msg, k, c->prng_partitionable, mk);
    Msg m;
    m.type = d[0];
    m.side = d[0] == 4 ? wsub(0, d[1]) : d[1];
    m.price = d[3]; m.qty = d[2]; m.oid = d[4]; m.tid = d[5]; m.t = d[6]; m.tns = d[7];
    i32 s = m.side, t = m.type;
    int lim = (t == 1) || (t == 4), cnl = (t == 2) || (t == 3);
    int index = (s == 1 && lim) * 1 + (s == -1 && cnl) * 2 + (s == 1 && cnl) * 3 + (s == 0 && t == 0) * 4;
#ifdef ORACLE_STATS
    STAT(index);
    if (t == 4) STAT(5);
    if ((index == 0 || index == 1) && m.qty <= 0) STAT(6);
    long long before = oracle_stats[20];
    i32 ba0[2], bb0[2], ba1[2], bb1[2];
    best_quotes(c, asks, bids, ba0, bb0);
    /* the message's class for the stats trace (tools/msg_mix.py): only the stats build pays these
       O(nOrders) scans; the checker and the CPU baseline skip them */
    int cls = -1;
    if (index == 4) cls = 0;
    else if (index >= 2) {
        const i32* sd = index == 2 ? asks : bids;
        int nO = c->n_orders, idx = -1;
        for (int i = 0; i < nO; ++i)
            if (sd[i * 6 + 2] == m.oid) { idx = i; break; }
        if (m.qty == 0) cls = 5;
        else if (idx >= 0) cls = 6;
        else {
            i32 lo = wsub(c->init_id, wmul(c->book_depth, 2));
            for (int i = 0; i < nO; ++i) {
                const i32* r = sd + i * 6;
                if (r[0] == m.price && r[2] <= c->init_id && r[2] >= lo && r[1] >= m.qty) { idx = i; break; }
            }
            cls = idx >= 0 ? 7 : (sd[(nO - 1) * 6] == -1 ? 8 : 9);
            if (cls == 8) /* an init-id row at the price, but with a smaller quantity (10) */
                for (int i = 0; i < nO; ++i) {
                    const i32* r = sd + i * 6;
                    if (r[0] == m.price && r[2] <= c->init_id && r[2] >= lo) { cls = 10; break; }
                }
        }
    } else {
        const i32* own = index == 1 ? bids : asks;
        int nO = c->n_orders, full = 1;
        for (int i = 0; i < nO; ++i) full &= own[i * 6] >= 0;
        cls = full ? 4 : 1;
    }
#endif
    switch (index) {
        case 0: ask_lim(c, m, asks, bids, trades); break;
        case 1: bid_lim(c, m, asks, bids, trades); break;
        case 2: cancel_order(c, asks, &m, mk); break;
        case 3: cancel_order(c, bids, &m, mk); break;
        default: break; /* doNothing */
    }
#ifdef ORACLE_STATS
    if ((index == 0 || index == 1) && oracle_stats[20] > before) STAT(7);   /* crossing */
    best_quotes(c, asks, bids, ba1, bb1);
    if (cls == 1 && oracle_stats[20] > before) cls = 3;
    else if (cls == 1 && (index == 1 ? bb1[0] != bb0[0] : ba1[0] != ba0[0])) cls = 2;
    if (oracle_trace_n < (1 << 24)) oracle_trace[oracle_trace_n++] = (signed char)cls;
    if (ba1[0] != ba0[0]) STAT(15);
    if (bb1[0] != bb0[0]) STAT(16);
    if (ba1[0] != ba0[0] || ba1[1] != ba0[1]) STAT(17);
    if (bb1[0] != bb0[0] || bb1[1] != bb0[1]) STAT(18);
#endif
}

static int lob_cfg_ok(const hftlob_lob_cfg* c) {
    return c->cancel_mode >= 0 && c->cancel_mode <= 3 && c->type_4_interpretation >= 0 &&
           c->type_4_interpretation <= 2 && c->n_orders > 0 && c->n_orders <= HFTLOB_MAX_SLOTS &&
           c->n_trades > 0 && c->n_trades <= HFTLOB_MAX_SLOTS;
}

/* scan_through_entire_array[_save_bidask] — :736-823, batched over envs (host memory) */
int oracle_book_process(const hftlob_lob_cfg* c, int n_env, int n_msg, const u32* keys, const i32* msgs, i32* asks,
                        i32* bids, i32* trades, i32* best_asks, i32* best_bids) {
    if (!lob_cfg_ok(c)) return HFTLOB_EINVAL;
    if (c->cancel_mode >= 2 && !keys) return HFTLOB_ENULL;
    int nO = c->n_orders, nT = c->n_trades;
#pragma omp parallel for schedule(dynamic, 16)
    for (int e = 0; e < n_env; ++e) {
        i32 *a = asks + (size_t)e * nO * 6, *b = bids + (size_t)e * nO * 6, *tr = trades + (size_t)e * nT * 8;
        for (int k = 0; k < n_msg; ++k) {
            process_msg(c, msgs + ((size_t)e * n_msg + k) * 8, a, b, tr, keys ? keys + 2 * e : NULL, n_msg, k);
            if (best_asks)
                best_quotes(c, a, b, best_asks + ((size_t)e * n_msg + k) * 2, best_bids + ((size_t)e * n_msg + k) * 2);
        }
    }
    return HFTLOB_OK;
}

/* getCancelMsgs — :827-853: first `size` slots with tid == agent, padded with
 * the appended all-zero row */
static void get_cancel_msgs(const i32* s, int nO, i32 agent, int size, i32 side, i32 t, i32 tns, i32* out) {
    int n = 0;
    for (int i = 0; i < nO && n < size; ++i)
        if (s[i * 6 + 3] == agent) {
            i32* o = out + n * 8;
            o[0] = 2; o[1] = side; o[2] = s[i * 6 + 1]; o[3] = s[i * 6]; o[4] = s[i * 6 + 2];
            o[5] = s[i * 6 + 3]; o[6] = t; o[7] = tns;
            ++n;
        }
    for (; n < size; ++n) {
        i32* o = out + n * 8;
        o[0] = 2; o[1] = side; o[2] = 0; o[3] = 0; o[4] = 0; o[5] = 0; o[6] = t; o[7] = tns;
    }
}

/* _filter_messages — mm_env.py:520-582 == exec_env.py:413-475 */
static void filter_messages(i32* act, i32* cnl, int n) {
    int am[HFTLOB_MAX_MSGS], cm[HFTLOB_MAX_MSGS];
    for (int i = 0; i < n; ++i) { am[i] = 0; cm[i] = 0; }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            if (cnl[j * 8 + 3] == act[i * 8 + 3] && act[i * 8 + 3] != 0) { am[i] = 1; cm[j] = 1; }
    i32 a[HFTLOB_MAX_MSGS], c[HFTLOB_MAX_MSGS], rel[HFTLOB_MAX_MSGS];
    int k = 0;
    for (int i = 0; i < n; ++i) if (am[i]) a[k++] = act[i * 8 + 2];
    for (; k < n; ++k) a[k] = 0;
    k = 0;
    for (int j = 0; j < n; ++j) if (cm[j]) c[k++] = cnl[j * 8 + 2];
    for (; k < n; ++k) c[k] = 0;
    for (int i = 0; i < n; ++i) rel[i] = (c[i] >= a[i]) ? a[i] : 0;
    /* rank_rev(mask)[i]: position of i in the descending, left-to-right-stable order */
    int na = 0, nc = 0;
    for (int i = 0; i < n; ++i) { na += am[i]; nc += cm[i]; }
    int ta = 0, fa = 0, tc = 0, fc = 0;
    for (int i = 0; i < n; ++i) {
        int r = am[i] ? ta++ : na + fa++;
        act[i * 8 + 2] = wsub(act[i * 8 + 2], rel[r]);
        if (act[i * 8 + 2] == 0) for (int f = 0; f < 8; ++f) act[i * 8 + f] = 0;
        int rc = cm[i] ? tc++ : nc + fc++;
        cnl[i * 8 + 2] = wsub(cnl[i * 8 + 2], rel[rc]);
    }
}

/* ============================================================ env helpers */
typedef struct {
    const hftlob_env_cfg* c;
    i32* rec;
} Env;

#define ASKS(E) ((E)->rec + (E)->c->off_asks)
#define BIDS(E) ((E)->rec + (E)->c->off_bids)
#define TRADES(E) ((E)->rec + (E)->c->off_trades)
#define LOADED(E) ((E)->rec + (E)->c->off_loaded)
#define BBIDS(E) ((E)->rec + (E)->c->off_best_bids)
#define BASKS(E) ((E)->rec + (E)->c->off_best_asks)
#define WORLD(E) ((E)->rec + (E)->c->off_world)
/* loaded: 0,1 init_time; 2 window_index; 3 max_steps; 4 start_index; 5 step_counter
 * world : 0,1 time; 2 order_id_counter; 3 mid_price(f); 4 delta_time(f) */

static int agent_words(const hftlob_agent_type_cfg* t) { return t->kind == HFTLOB_AGENT_MM ? 5 : 13; }

/* MM state words: 0 posted_distance_bid 1 posted_distance_ask 2 inventory 3 total_PnL(f) 4 cash(f)
 * EXE state words: 0 init_price(f) 1 task 2 qexec 3 is_sell 4 p_vwap 5 total_revenue 6 drift_return
 *   7 advantage_return 8 slippage_rm 9 price_adv_rm 10 price_drift_rm 11 vwap_rm 12 trade_duration */

/* get_best_ask / get_best_bid (no quantities) on a side masked by tid != trader */
static void masked_best(const hftlob_env_cfg* c, const i32* asks, const i32* bids, i32 tid, i32* ba, i32* bb) {
    int nO = c->lob.n_orders;
    i32 mn = c->lob.maxint, mx = INT32_MIN;
    for (int i = 0; i < nO; ++i) {
        i32 pa = asks[i * 6 + 3] != tid ? asks[i * 6] : -1;
        i32 pb = bids[i * 6 + 3] != tid ? bids[i * 6] : -1;
        mn = imin(mn, pa == -1 ? c->lob.maxint : pa);
        mx = imax(mx, pb);
    }
    *ba = mn == c->lob.maxint ? -1 : mn;
    *bb = mx;
}

/* get_volume — :919-930 */
static i32 side_volume(const i32* s, int nO) {
    i32 v = 0;
    for (int i = 0; i < nO; ++i) if (s[i * 6] != -1) v = wadd(v, s[i * 6 + 1]);
    return v;
}

typedef struct { /* per-agent action extras */
    i32 bid_price, ask_price, bid_dist, ask_dist, bid_quant, ask_quant, empty_book;
} ActX;

/* MM _getActionMsgs_fixedQuant — mm_env.py:970-1118 */
static void mm_fixed_quant(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st,
                           i32 tid, i32 action, i32* out, ActX* x) {
    static const float boff[10] = {0, 1, 2, 3, 4, 0, 2, 5, 1, 0};
    static const float aoff[10] = {0, 1, 2, 3, 4, 2, 0, 1, 5, 0};
    static const i32 bq[10] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 0};
    static const i32 aq[10] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 0};
    if (tc->fixed_action_setting) action = tc->fixed_action;
    i32 tick = c->tick_size;
    i32 ba, bb;
    masked_best(c, ASKS(E), BIDS(E), tid, &ba, &bb);
    int empty = (ba == -1) || (bb == -1);
    ba = wmul(ifloordiv(ba, tick), tick);
    bb = wmul(ifloordiv(bb, tick), tick);
    if (empty) { bb = BBIDS(E)[(c->n_msgs - 1) * 2]; ba = BASKS(E)[(c->n_msgs - 1) * 2]; }
    float hsp = fmaxf(i2f(wsub(ba, bb)) / 2.0f, (float)tick / 2.0f);
    float hs = (ffloordiv(hsp, (float)tick) + 1.0f) * (float)tick;
    float bo, ao;
    i32 bquant, aquant;
    if (!tc->sell_buy_all_option) {
        int ai = gather_idx(action, 10); /* jnp gather: negative wraps, then clamps */
        bo = boff[ai]; ao = aoff[ai];
        bquant = wmul(bq[ai], tc->fixed_quant_value); aquant = wmul(aq[ai], tc->fixed_quant_value);
    } else { /* mm_env.py:1018-1023 */
        static const float boff9[9] = {10, 2, 4, -1, 0, 2, -20, 0, 0};
        static const float aoff9[9] = {10, 2, 4, -1, 2, 0, 0, -20, 0};
        i32 iq = ifloordiv(st[2], tc->fixed_quant_value);
        i32 bq9[9] = {1, 1, 1, 1, 1, 1, iq, 0, 0}, aq9[9] = {1, 1, 1, 1, 1, 1, 0, iq, 0};
        int ai = gather_idx(action, 9);
        bo = boff9[ai]; ao = aoff9[ai];
        bquant = wmul(bq9[ai], tc->fixed_quant_value); aquant = wmul(aq9[ai], tc->fixed_quant_value);
    }
    if (empty) { bquant = 0; aquant = 0; }
    float bpf = i2f(bb) - bo * hs;
    float apf = i2f(ba) + ao * hs;
    i32 bp = f2i(ffloordiv(fmaxf(bpf, 0.0f), (float)tick) * (float)tick);
    i32 ap = f2i(ffloordiv(fmaxf(i2f(wadd(bp, tick)), apf), (float)tick) * (float)tick);
    i32 typ[2] = {1, 1}, sd[2] = {1, -1}, q[2] = {bquant, aquant}, p[2] = {bp, ap};
    i32 inv = st[2];
    i32 lq[2] = {f2i(tc->auto_liquidate_alpha * i2f(imax(wsub(0, inv), 0))),
                 f2i(tc->auto_liquidate_alpha * i2f(imax(inv, 0)))};
    i32 lp[2] = {f2i(i2f(ba) + hs * 10.0f), f2i(i2f(bb) - hs * 10.0f)};
    if (tc->tenth_action_market && action == 9) {
        for (int k = 0; k < 2; ++k) { typ[k] = 4; sd[k] = k == 0 ? -1 : 1; q[k] = lq[k]; p[k] = lp[k]; }
    }
    if (tc->auto_liquidate_threshold != 0 && iabs(inv) > tc->auto_liquidate_threshold) {
        for (int k = 0; k < 2; ++k) { typ[k] = 4; sd[k] = k == 0 ? -1 : 1; q[k] = lq[k]; p[k] = lp[k]; }
    }
    const i32* wt = WORLD(E);
    for (int k = 0; k < 2; ++k) {
        i32* o = out + k * 8;
        o[0] = typ[k]; o[1] = sd[k]; o[2] = q[k]; o[3] = p[k]; o[4] = c->placeholder_order_id; o[5] = tid;
        o[6] = wadd(wt[0], tc->time_delay_obs_act); o[7] = wadd(wt[1], tc->time_delay_obs_act);
    }
    x->bid_price = bp; x->ask_price = ap; x->bid_dist = wsub(bb, bp); x->ask_dist = wsub(ap, ba);
    x->bid_quant = bquant; x->ask_quant = aquant; x->empty_book = empty;
}

/* MM bobRL (:1474-1561), bobStrategy (:1400-1472), AvSt (:1248-1398),
 * spread_skew (:1667-1808), simple (:1123-1246) */
static void mm_other_actions(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st, i32 tid,
                             i32 action, i32* out, ActX* x) {
    static const i32 bob1b[3] = {1, 2, 0}, bob1a[3] = {1, 0, 2};
    static const i32 bob2b[5] = {2, 3, 1, 4, 0}, bob2a[5] = {2, 1, 3, 0, 4};
    static const i32 bob5b[11] = {5, 6, 4, 7, 3, 8, 2, 9, 1, 10, 0}, bob5a[11] = {5, 4, 6, 3, 7, 2, 8, 1, 9, 0, 10};
    static const i32 bob10b[21] = {10, 11, 9, 12, 8, 13, 7, 14, 6, 15, 5, 16, 4, 17, 3, 18, 2, 19, 1, 20, 0};
    static const i32 bob10a[21] = {10, 9, 11, 8, 12, 7, 13, 6, 14, 5, 15, 4, 16, 3, 17, 2, 18, 1, 19, 0, 20};
    static const float gammas[8] = {0.1f, 0.2f, 0.5f, 1.0f, 2.0f, 5.0f, 10.0f, 20.0f};
    if (tc->fixed_action_setting) action = tc->fixed_action;
    i32 tick = c->tick_size, inv = st[2], fq = tc->fixed_quant_value;
    i32 lba = BASKS(E)[(c->n_msgs - 1) * 2], lbb = BBIDS(E)[(c->n_msgs - 1) * 2];
    i32 bp = 0, ap = 0, bq = 0, aq = 0;
    x->bid_price = x->ask_price = x->bid_dist = x->ask_dist = 0;
    x->empty_book = 0;
    int kind = tc->action_space;
    if (kind == HFTLOB_MM_ACT_BOB_RL || kind == HFTLOB_MM_ACT_BOB_STRATEGY || kind == HFTLOB_MM_ACT_AVST) {
        i32 ba, bb;
        masked_best(c, ASKS(E), BIDS(E), tid, &ba, &bb);
        int empty = (ba == -1) || (bb == -1);
        ba = wmul(ifloordiv(ba, tick), tick);
        bb = wmul(ifloordiv(bb, tick), tick);
        if (empty) { bb = lbb; ba = lba; }
        if (kind == HFTLOB_MM_ACT_BOB_RL) {
            const i32 *tb, *ta;
            int n;
            switch (tc->bob_v0) {
                case 1: tb = bob1b; ta = bob1a; n = 3; break;
                case 2: tb = bob2b; ta = bob2a; n = 5; break;
                case 5: tb = bob5b; ta = bob5a; n = 11; break;
                default: tb = bob10b; ta = bob10a; n = 21; break;
            }
            int i = gather_idx(action, n);
            bq = empty ? 0 : wmul(tb[i], fq);
            aq = empty ? 0 : wmul(ta[i], fq);
            bp = bb; ap = ba;
        } else if (kind == HFTLOB_MM_ACT_BOB_STRATEGY) {
            float kappa = i2f(wadd(action, 1)) / i2f(wmul(tc->bob_v0, 5));
            float v0 = (float)tc->bob_v0;
            bq = f2i_sat(rintf(v0 * fmaxf(1.0f - kappa * i2f(inv), 0.0f)));
            aq = f2i_sat(rintf(v0 * fmaxf(1.0f + kappa * i2f(inv), 0.0f)));
            if (empty) bq = aq = 0;
            bp = bb; ap = ba;
        } else {
            i32 mid = ifloordiv(wadd(ba, bb), 2);
            int i = gather_idx(action, 8);
            float gamma = gammas[i];
            const i32* L = LOADED(E);
            i32 tl = c->ep_type == 1 ? wsub(c->episode_time, wsub(WORLD(E)[0], L[0])) : wsub(c->episode_time, L[5]);
            float nt = i2f(tl) / i2f(c->episode_time);
            float res = i2f(mid) - i2f(inv) * gamma * tc->avst_var * nt;
            float spread = gamma * tc->avst_var * nt + (2.0f / gamma) * tc->avst_log_term[i];
            spread = fminf(fmaxf(spread, (float)tick), (float)c->lob.maxint);
            float bf = fminf(fmaxf(res - spread / 2.0f, 0.0f), (float)c->lob.maxint);
            float af = fminf(fmaxf(res + spread / 2.0f, 0.0f), (float)c->lob.maxint);
            bp = f2i_sat(ffloordiv(bf, (float)tick) * (float)tick);
            ap = f2i_sat(ffloordiv(af, (float)tick) * (float)tick);
            i32 q = ifloordiv(mid, tick), m = wsub(mid, wmul(q, tick));
            i32 rdown = wmul(wsub(q, m == 0 ? 1 : 0), tick), rup = wmul(wadd(q, 1), tick);
            bp = imin(bp, rdown);
            ap = imax(ap, rup);
            bq = aq = fq;
            x->bid_price = bp; x->ask_price = ap; x->bid_dist = wsub(bb, bp); x->ask_dist = wsub(ap, ba);
        }
        if (kind != HFTLOB_MM_ACT_AVST) x->empty_book = empty;
    } else {
        i32 ba = wmul(ifloordiv(lba, tick), tick), bb = wmul(ifloordiv(lbb, tick), tick);
        if (kind == HFTLOB_MM_ACT_SPREAD_SKEW) {
            float mid = i2f(wadd(ba, bb)) / 2.0f;
            i32 cur = wsub(ba, bb);
            i32 stype = ifloordiv(action, 3), skew = wsub(action, wmul(stype, 3));
            float mult = stype == 0 ? 1.0f : tc->spread_multiplier;
            float nsp = i2f(cur) * mult;
            float skt = skew == 0 ? -tc->skew_multiplier : (skew == 1 ? 0.0f : tc->skew_multiplier);
            float smid = tc->multiplier_type ? mid + skt * nsp : mid + skt * (float)tick;
            float hs = ffloordiv(nsp, 2.0f);
            bp = f2i_sat(ffloordiv(smid - hs, (float)tick) * (float)tick);
            ap = f2i_sat(ffloordiv(smid + hs, (float)tick) * (float)tick);
            bq = aq = fq;
        } else {
            static const float boffs[4] = {0, -2000, 0, 0}, aoffs[4] = {0, 0, -2000, 0};
            int n = tc->simple_nothing_action ? 4 : 3;
            int i = gather_idx(action, n);
            if (tc->sell_buy_all_option) {
                i32 bqa, aqa;
                if (inv > 0) { bqa = fq; aqa = imax(iabs(inv), fq); }
                else { bqa = imax(iabs(inv), fq); aqa = fq; }
                i32 tbq[4] = {fq, bqa, 0, 0}, taq[4] = {fq, 0, aqa, 0};
                bq = tbq[i]; aq = taq[i];
            } else {
                static const i32 tbq[4] = {1, 1, 0, 0}, taq[4] = {1, 0, 1, 0};
                bq = wmul(tbq[i], fq); aq = wmul(taq[i], fq);
            }
            float to = (float)wmul(tc->n_ticks_offset, tick);
            float bf = i2f(bb) - boffs[i] * to, af = i2f(ba) + aoffs[i] * to;
            bp = f2i_sat(ffloordiv(fmaxf(bf, 0.0f), (float)tick) * (float)tick);
            ap = f2i_sat(ffloordiv(af, (float)tick) * (float)tick);
        }
    }
    i32 q[2] = {bq, aq}, p[2] = {bp, ap}, sd[2] = {1, -1};
    const i32* wt = WORLD(E);
    for (int k = 0; k < 2; ++k) {
        i32* o = out + k * 8;
        o[0] = 1; o[1] = sd[k]; o[2] = q[k]; o[3] = p[k]; o[4] = c->placeholder_order_id; o[5] = tid;
        o[6] = wadd(wt[0], tc->time_delay_obs_act); o[7] = wadd(wt[1], tc->time_delay_obs_act);
    }
    x->bid_quant = bq; x->ask_quant = aq;
}

/* MM _getActionMsgs_directional_trading — mm_env.py:1810-1865 */
static void mm_directional(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, i32 tid, i32 action,
                           i32* out, ActX* x) {
    i32 tick = c->tick_size;
    i32 ba = wmul(ifloordiv(BASKS(E)[(c->n_msgs - 1) * 2], tick), tick);
    i32 bb = wmul(ifloordiv(BBIDS(E)[(c->n_msgs - 1) * 2], tick), tick);
    int ai = gather_idx(action, 3);
    i32 bq = (ai == 1) * tc->fixed_quant_value, aq = (ai == 2) * tc->fixed_quant_value;
    i32 q[2] = {bq, aq}, p[2] = {ba, bb}, sd[2] = {1, -1};
    const i32* wt = WORLD(E);
    for (int k = 0; k < 2; ++k) {
        i32* o = out + k * 8;
        o[0] = 1; o[1] = sd[k]; o[2] = q[k]; o[3] = p[k]; o[4] = c->placeholder_order_id; o[5] = tid;
        o[6] = wadd(wt[0], tc->time_delay_obs_act); o[7] = wadd(wt[1], tc->time_delay_obs_act);
    }
    memset(x, 0, sizeof *x);
    x->bid_quant = bq; x->ask_quant = aq;
}

/* EXE _getActionMsgs_fixedQuant_extended — exec_env.py:838-932 */
static void exe_fqc(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st, i32 tid,
                    i32 action, i32* out) {
    static const i32 QA[13][4] = {{0, 0, 0, 0}, {1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1},
                                  {2, 0, 0, 0}, {0, 2, 0, 0}, {0, 0, 2, 0}, {0, 0, 0, 2}, {5, 0, 0, 0},
                                  {0, 5, 0, 0}, {0, 0, 5, 0}, {0, 0, 0, 5}};
    i32 tick = c->tick_size;
    i32 ba = wmul(ifloordiv(BASKS(E)[(c->n_msgs - 1) * 2], tick), tick);
    i32 bb = wmul(ifloordiv(BBIDS(E)[(c->n_msgs - 1) * 2], tick), tick);
    i32 sell = st[3];
    i32 pl[4];
    if (sell) {
        pl[0] = bb;
        pl[1] = f2i(ceilf(ffloordiv(i2f(wadd(bb, ba)) / 2.0f, (float)tick)) * (float)tick);
        pl[2] = ba;
        pl[3] = wadd(ba, wmul(tick, tc->n_ticks_in_book));
    } else {
        pl[0] = ba;
        pl[1] = wmul(ifloordiv(ifloordiv(wadd(bb, ba), 2), tick), tick);
        pl[2] = bb;
        pl[3] = wsub(bb, wmul(tick, tc->n_ticks_in_book));
    }
    i32 fq = tc->fixed_quant_value, left = wsub(st[1], st[2]);
    i32 q[4] = {0, 0, 0, 0}, p[4] = {pl[0], pl[1], pl[2], pl[3]};
    int n = 4;
    switch (tc->action_space) {
        case HFTLOB_EXE_ACT_FIXED_QUANTS_COMPLEX: { /* :838-933 */
            int ai = gather_idx(action, 13);
            i32 tot = 0;
            for (int k = 0; k < 4; ++k) { q[k] = wmul(QA[ai][k], fq); tot = wadd(tot, q[k]); }
            if (!(tot <= left)) { q[0] = f2i(floorf(i2f(left))); q[1] = q[2] = q[3] = 0; }
            break;
        }
        case HFTLOB_EXE_ACT_FIXED_QUANTS_1MSG: { /* :732-836: one message */
            static const i32 QN[5] = {0, 1, 1, 1, 1};
            int ai = gather_idx(action, 5);
            i32 prices[5] = {0, pl[0], pl[1], pl[2], pl[3]};
            i32 sq = wmul(QN[ai], fq);
            q[0] = sq <= left ? sq : 0;
            p[0] = prices[ai];
            n = 1;
            break;
        }
        case HFTLOB_EXE_ACT_SIMPLEST_CASE: { /* :935-999: (FT, NT) */
            int ai = gather_idx(action, 3);
            i32 QS[3][2] = {{0, 0}, {fq, 0}, {0, fq}};
            q[0] = QS[ai][0]; q[1] = QS[ai][1];
            if (!(wadd(q[0], q[1]) <= left)) { q[0] = f2i(floorf(i2f(wmul(QS[1][0], left)))); q[1] = 0; }
            p[0] = sell ? bb : ba; p[1] = sell ? ba : bb;
            n = 2;
            break;
        }
        default: { /* twap :1126-1227 (fixed_steps): ceil(max(left, 0) / steps_left) */
            static const i32 QT[2][2] = {{1, 0}, {0, 1}};
            const i32* L = LOADED(E);
            i32 steps_left = wsub(wsub(L[3], L[5]), 1);
            i32 qts = f2i_sat(ceilf(i2f(imax(left, 0)) / i2f(steps_left)));
            int ai = gather_idx(action, 2);
            q[0] = wmul(QT[ai][0], qts); q[1] = wmul(QT[ai][1], qts);
            p[0] = sell ? bb : ba; p[1] = sell ? ba : bb;
            n = 2;
            break;
        }
    }
    i32 side = wsub(1, wmul(sell, 2));
    const i32* wt = WORLD(E);
    for (int k = 0; k < n; ++k) {
        i32* o = out + k * 8;
        o[0] = 1; o[1] = side; o[2] = q[k]; o[3] = p[k]; o[4] = c->placeholder_order_id; o[5] = tid;
        o[6] = wadd(wt[0], tc->time_delay_obs_act); o[7] = wadd(wt[1], tc->time_delay_obs_act);
    }
}

/* EXE _getActionMsgs_fixedPrice — exec_env.py:1001-1123.  `action` holds n_actions
 * (1..4) quantities, one per price level. */
static void exe_fixed_price(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st, i32 tid,
                            const i32* action, i32* out) {
    int n = tc->n_actions;
    i32 tick = c->tick_size, left = wsub(st[1], st[2]), sell = st[3];
    /* :1005-1010: if sum(action) > left: (action / sum(action) * left).astype(int32) (f32) */
    i32 sum = 0, a[4];
    for (int k = 0; k < n; ++k) sum = wadd(sum, action[k]);
    for (int k = 0; k < n; ++k)
        a[k] = sum > left ? f2i_sat((float)action[k] / (float)sum * (float)left) : action[k];
    /* :1089-1090: best_asks[-10:].mean(axis=0)[0] // tick * tick, as int32 */
    int M = c->n_msgs, lo = M > 10 ? M - 10 : 0;
    float ma = 0.0f, mb = 0.0f;
    for (int m = lo; m < M; ++m) { ma += (float)BASKS(E)[m * 2]; mb += (float)BBIDS(E)[m * 2]; }
    ma /= (float)(M - lo);
    mb /= (float)(M - lo);
    i32 best_ask = f2i_sat(ffloordiv(ma, (float)tick) * (float)tick);
    i32 best_bid = f2i_sat(ffloordiv(mb, (float)tick) * (float)tick);
    /* buy_task_prices / sell_task_prices :1043-1076 -> (FT, M, NT, PP, MKT) */
    i32 FT, Mp, NT, PP, MKT;
    if (sell) {
        FT = wmul(ifloordiv(best_bid, tick), tick);
        Mp = f2i_sat(ceilf(ffloordiv((float)wadd(best_bid, best_ask) / 2.0f, (float)tick)) * (float)tick);
        NT = best_ask;
        PP = wadd(best_ask, wmul(tick, tc->n_ticks_in_book));
        MKT = 0;
    } else {
        FT = wmul(ifloordiv(best_ask, tick), tick);
        Mp = wmul(ifloordiv(ifloordiv(wadd(best_bid, best_ask), 2), tick), tick);
        NT = best_bid;
        PP = wsub(best_bid, wmul(tick, tc->n_ticks_in_book));
        MKT = c->lob.maxint;
    }
    i32 levels[5];
    int nl = 0;
    levels[nl++] = FT;
    if (n == 4) levels[nl++] = Mp;
    if (n >= 2) levels[nl++] = NT;
    if (n >= 3) levels[nl++] = PP;
    levels[nl++] = MKT;
    /* normal_quant_price :1013-1033: prices = price_levels[:-1]; n == 4 and M == NT: merge into NT */
    i32 q[4], p[4];
    for (int k = 0; k < n; ++k) { q[k] = a[k]; p[k] = levels[k]; }
    if (n == 4 && levels[1] == levels[2]) {
        q[2] = wadd(q[2], q[1]);
        q[1] = 0;
        p[1] = -1;
    }
    i32 side = wsub(1, wmul(sell, 2));
    const i32* wt = WORLD(E);
    for (int k = 0; k < n; ++k) {
        i32* o = out + k * 8;
        o[0] = 1; o[1] = side; o[2] = q[k]; o[3] = p[k]; o[4] = c->placeholder_order_id; o[5] = tid;
        o[6] = wadd(wt[0], tc->time_delay_obs_act); o[7] = wadd(wt[1], tc->time_delay_obs_act);
    }
}

/* ---- trade-log helpers for rewards */
/* add_trade — JaxOrderBookArrays.py:885-889: first row holding ANY -1 field */
static void add_trade(i32* tr, int nT, const i32* row) {
    int idx = nT - 1;
    for (int i = 0; i < nT * 8; ++i)
        if (tr[i] == -1) { idx = i / 8; break; }
    memcpy(tr + idx * 8, row, 8 * sizeof(i32));
}

typedef struct {
    float reward, reward_pv, reward_spooner, end_of_ep_pv, reward_spooner_damped, reward_spooner_asym_damped,
        reward_spooner_asym_damped2, reward_delta_pv, market_share, delta_mid, buyPnL, sellPnL, invPnL, PnL,
        cash, inventoryValue;
    i32 end_inventory, forced_unwind;
} MMRew;

/* MM get_reward — mm_env.py:2214-2673 */
static void mm_reward(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st, i32 tid,
                      const i32* trades_in, const i32* bba, const i32* bbb, int ep_done, MMRew* R) {
    int nT = c->lob.n_trades, M = c->n_msgs;
    float tick = (float)c->tick_size;
    i32 tr[HFTLOB_MAX_SLOTS * 8];
    memcpy(tr, trades_in, (size_t)nT * 8 * sizeof(i32));
    i32 inv = st[2];
    /* pre-unwind buy/sell quantities */
    i32 bqs = 0, sqs = 0;
    for (int i = 0; i < nT; ++i) {
        const i32* r = tr + i * 8;
        if (r[0] < 0) continue;
        if (!(r[6] == tid || r[7] == tid)) continue;
        int buy = (r[1] >= 0 && r[6] == tid) || (r[1] < 0 && r[7] == tid);
        int sel = (r[1] < 0 && r[6] == tid) || (r[1] >= 0 && r[7] == tid);
        if (buy) bqs = wadd(bqs, iabs(r[1]));
        if (sel) sqs = wadd(sqs, iabs(r[1]));
    }
    i32 inv_b = wsub(wadd(inv, bqs), sqs);
    float mids[HFTLOB_MAX_MSGS];
    for (int m = 0; m < M; ++m) mids[m] = i2f(wadd(bbb[m * 2], bba[m * 2])) / 2.0f;
    float avg_mid = wsum(mids, M) / (float)M;
    float last_mid = i2f(wadd(bbb[(M - 1) * 2], bba[(M - 1) * 2])) / 2.0f;
    i32 pen = wmul(tc->unwind_price_penalty, c->tick_size);
    pen = inv_b > 0 ? pen : wsub(0, pen);
    i32 unwind_px; /* far_touch stays int32 in the reference; mid / mid_avg are f32 */
    if (tc->unwind_price == HFTLOB_PRICE_FAR_TOUCH)
        unwind_px = wsub(inv_b > 0 ? bbb[(M - 1) * 2] : bba[(M - 1) * 2], pen);
    else
        unwind_px = f2i((tc->unwind_price == HFTLOB_PRICE_MID_AVG ? avg_mid : last_mid) - i2f(pen));
    if (ep_done && iabs(inv_b) > 0) {
        i32 row[8] = {unwind_px, wmul(isign(inv_b), iabs(inv_b)), c->artificial_order_id,
                      c->placeholder_order_id, 0, 0, c->artificial_trader_id, tid};
        add_trade(tr, nT, row);
    }
    R->forced_unwind = wmul(inv_b, ep_done);
    /* post-unwind stats */
    float mid_end = last_mid;
    float inc[HFTLOB_MAX_SLOTS], out[HFTLOB_MAX_SLOTS], rb[HFTLOB_MAX_SLOTS], rs[HFTLOB_MAX_SLOTS];
    float bpl[HFTLOB_MAX_SLOTS], spl[HFTLOB_MAX_SLOTS], abp[HFTLOB_MAX_SLOTS], asp[HFTLOB_MAX_SLOTS];
    i32 bq = 0, sq = 0, oq = 0;
    i32 bP[HFTLOB_MAX_SLOTS], bQ[HFTLOB_MAX_SLOTS], sP[HFTLOB_MAX_SLOTS], sQ[HFTLOB_MAX_SLOTS];
    i32 pbP[HFTLOB_MAX_SLOTS], pbQ[HFTLOB_MAX_SLOTS], psP[HFTLOB_MAX_SLOTS], psQ[HFTLOB_MAX_SLOTS];
    for (int i = 0; i < nT; ++i) {
        const i32* r = tr + i * 8;
        int valid = r[0] >= 0;
        i32 P = valid ? r[0] : 0, Q = valid ? r[1] : 0, pt = valid ? r[6] : 0, at = valid ? r[7] : 0;
        int mine = (tid == pt) || (tid == at);
        i32 aP = mine ? P : 0, aQ = mine ? Q : 0, apt = mine ? pt : 0, aat = mine ? at : 0;
        if (!mine) oq = wadd(oq, iabs(Q));
        int buy = (aQ >= 0 && tid == apt) || (aQ < 0 && tid == aat);
        int sel = (aQ < 0 && tid == apt) || (aQ >= 0 && tid == aat);
        int pbuy = (aQ >= 0 && tid == apt), psel = (aQ < 0 && tid == apt);
        bP[i] = buy ? aP : 0; bQ[i] = buy ? aQ : 0; sP[i] = sel ? aP : 0; sQ[i] = sel ? aQ : 0;
        pbP[i] = pbuy ? aP : 0; pbQ[i] = pbuy ? aQ : 0; psP[i] = psel ? aP : 0; psQ[i] = psel ? aQ : 0;
        bq = wadd(bq, iabs(bQ[i]));
        sq = wadd(sq, iabs(sQ[i]));
    }
    for (int i = 0; i < nT; ++i) {
        inc[i] = i2f(sP[i]) / tick * i2f(iabs(sQ[i]));
        out[i] = i2f(bP[i]) / tick * i2f(iabs(bQ[i]));
        rb[i] = i2f(pbP[i]) / tick * i2f(iabs(pbQ[i]));
        rs[i] = i2f(psP[i]) / tick * i2f(iabs(psQ[i]));
    }
    float income = wsum(inc, nT), outgoing = wsum(out, nT);
    i32 new_inv = wsub(wadd(inv, bq), sq);
    float rebate_value = wsum(rb, nT) + wsum(rs, nT);
    float rebate_income = rebate_value * tc->rebate_factor;
    float ref_buy, ref_sell, ref;
    int ref_int = tc->reference_price == HFTLOB_PRICE_FAR_TOUCH || tc->reference_price == HFTLOB_PRICE_NEAR_TOUCH;
    i32 rbi = 0, rsi = 0, refi = 0; /* touch prices are int32 in the reference */
    if (tc->reference_price == HFTLOB_PRICE_MID_AVG) { ref_buy = ref_sell = ref = avg_mid; }
    else if (ref_int) {
        int far = tc->reference_price == HFTLOB_PRICE_FAR_TOUCH;
        rbi = far ? bba[(M - 1) * 2] : bbb[(M - 1) * 2];
        rsi = far ? bbb[(M - 1) * 2] : bba[(M - 1) * 2];
        refi = new_inv > 0 ? rbi : rsi;
        ref_buy = i2f(rbi); ref_sell = i2f(rsi); ref = i2f(refi);
    } else { ref_buy = ref_sell = ref = last_mid; }
    float PnL = income - outgoing + rebate_income;
    float cash = bitf(st[4]) + PnL;
    float inv_value = ref_int ? i2f(wmul(new_inv, refi)) / tick : i2f(new_inv) * ref / tick;
    float net_worth = cash + inv_value;
    i32 traded = wadd(bq, sq);
    float market_share = i2f(traded) / i2f(wadd(traded, oq));
    const i32* wt = WORLD(E);
    float wmid = bitf(wt[3]);
    float invPnL = i2f(inv) * (mid_end - wmid) / tick;
    for (int i = 0; i < nT; ++i) {
        if (ref_int) {
            bpl[i] = i2f(wsub(rbi, bP[i])) / tick * i2f(iabs(bQ[i]));
            spl[i] = i2f(wsub(sP[i], rsi)) / tick * i2f(iabs(sQ[i]));
        } else {
            bpl[i] = (ref_buy - i2f(bP[i])) / tick * i2f(iabs(bQ[i]));
            spl[i] = (i2f(sP[i]) - ref_sell) / tick * i2f(iabs(sQ[i]));
        }
    }
    float buyPnL = wsum(bpl, nT), sellPnL = wsum(spl, nT);
    float eta = tc->inventoryPnL_eta, gam = tc->inventoryPnL_gamma;
    float r_sp = buyPnL + sellPnL + rebate_income + invPnL;
    float r_spd = buyPnL + sellPnL + rebate_income + invPnL - eta * invPnL;
    float r_spad = buyPnL + sellPnL + rebate_income + invPnL - fmaxf(0.0f, eta * invPnL);
    float r_spad2 = buyPnL + sellPnL + rebate_income + gam * (invPnL - fmaxf(0.0f, eta * invPnL));
    float r_sps = buyPnL + sellPnL + rebate_income + eta * (invPnL - tc->one_minus_eta * fmaxf(0.0f, invPnL));
    /* complex */
    i32 inv_change = wsub(bq, sq);
    for (int i = 0; i < nT; ++i) {
        abp[i] = i2f(bP[i]) / i2f(bq) * i2f(iabs(bQ[i]));
        asp[i] = i2f(sP[i]) / i2f(sq) * i2f(iabs(sQ[i]));
    }
    float avg_buy = bq > 0 ? wsum(abp, nT) : 0.0f;
    float avg_sell = sq > 0 ? wsum(asp, nT) : 0.0f;
    float real_pnl = i2f(imin(bq, sq)) * (avg_sell - avg_buy);
    float unreal_pnl = inv_change > 0 ? i2f(inv_change) * (avg_mid - avg_buy)
                                      : i2f(iabs(inv_change)) * (avg_sell - avg_mid);
    float r_complex = real_pnl + tc->unrealizedPnL_lambda * unreal_pnl + eta * fminf(invPnL, invPnL * eta);
    float r_pv = i2f(new_inv) * (ref / tick) + cash;
    float old_ref;
    if (tc->reference_price == HFTLOB_PRICE_FAR_TOUCH)
        old_ref = i2f(inv > 0 ? BASKS(E)[(M - 1) * 2] : BBIDS(E)[(M - 1) * 2]);
    else if (tc->reference_price == HFTLOB_PRICE_NEAR_TOUCH)
        old_ref = i2f(inv > 0 ? BBIDS(E)[(M - 1) * 2] : BASKS(E)[(M - 1) * 2]);
    else old_ref = wmid;
    float old_nw = old_ref / tick * i2f(inv) + bitf(st[4]);
    float d_nw = net_worth - old_nw;
    float reward;
    switch (tc->reward_function) {
        case HFTLOB_MM_REW_PORTFOLIO_VALUE: reward = r_pv; break;
        case HFTLOB_MM_REW_BUY_SELL_PNL: reward = buyPnL + sellPnL; break;
        case HFTLOB_MM_REW_COMPLEX: reward = r_complex; break;
        case HFTLOB_MM_REW_ZERO_INV: reward = i2f(wsub(0, iabs(new_inv))); break;
        case HFTLOB_MM_REW_SPOONER: reward = r_sp; break;
        case HFTLOB_MM_REW_SPOONER_DAMPED: reward = r_spd; break;
        case HFTLOB_MM_REW_SPOONER_ASYM_DAMPED: reward = r_spad; break;
        case HFTLOB_MM_REW_SPOONER_SCALED: reward = r_sps; break;
        case HFTLOB_MM_REW_DELTA_PORTFOLIO_VALUE: reward = d_nw; break;
        default: reward = r_spad2; break;
    }
    float inv_pen = 0.0f;
    if (tc->inv_penalty == HFTLOB_INVPEN_LINEAR) inv_pen = i2f(wsub(0, iabs(new_inv)));
    else if (tc->inv_penalty == HFTLOB_INVPEN_QUADRATIC)
        inv_pen = i2f(wmul(-1, wmul(new_inv, new_inv))) / tc->inv_penalty_quadratic_factor;
    else if (tc->inv_penalty == HFTLOB_INVPEN_THRESHOLD)
        inv_pen = i2f(iabs(new_inv)) > tc->inv_penalty_threshold
                      ? -1.0f * (i2f(wmul(new_inv, new_inv)) / tc->inv_penalty_quadratic_factor) : 0.0f;
    else if (tc->inv_penalty == HFTLOB_INVPEN_EXP4) /* mm_env.py:2528-2529 */
        inv_pen = -1.0f * expf(i2f(wmul(new_inv, 4)));
    reward = reward + tc->inv_penalty_lambda * inv_pen;
    if (tc->clip_reward) reward = fminf(fmaxf(reward, -10000.0f), 10000.0f);
    if (tc->volume_traded_bonus == 1) reward = reward + fabsf(reward) * market_share;
    if (tc->exclude_extreme_spreads) {
        int any = 0;
        for (int m = 0; m < M; ++m) {
            float spr = i2f(wsub(BASKS(E)[m * 2], BBIDS(E)[m * 2]));
            float mp = i2f(wadd(BASKS(E)[m * 2], BBIDS(E)[m * 2])) / 2.0f;
            any |= (spr / mp) > 0.1f;
        }
        if (any) reward = 0.0f;
    }
    R->reward = reward;
    R->reward_pv = r_pv;
    R->reward_spooner = r_sp;
    R->end_of_ep_pv = r_pv * (float)ep_done;
    R->reward_spooner_damped = r_spd;
    R->reward_spooner_asym_damped = r_spad;
    R->reward_spooner_asym_damped2 = r_spad2;
    R->reward_delta_pv = d_nw;
    R->market_share = market_share;
    R->delta_mid = mid_end - wmid;
    R->buyPnL = buyPnL;
    R->sellPnL = sellPnL;
    R->invPnL = invPnL;
    R->PnL = PnL;
    R->cash = cash;
    R->inventoryValue = inv_value;
    R->end_inventory = new_inv;
}

typedef struct {
    float reward, reward_info, p_vwap, vwap_rm, price_adv_rm, slippage_rm, price_drift_rm, advantage, drift,
        slippage, trade_duration;
    i32 agentQuant, qp_agent, doom_quant, quant_left;
} EXRew;

/* EXE get_reward — exec_env.py:1511-1762 */
static void exe_reward(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st, i32 tid,
                       const i32* trades_in, const i32* bba, const i32* bbb, int ep_done, EXRew* R) {
    int nT = c->lob.n_trades, M = c->n_msgs;
    i32 tick = c->tick_size;
    i32 tr[HFTLOB_MAX_SLOTS * 8];
    memcpy(tr, trades_in, (size_t)nT * 8 * sizeof(i32));
    i32 task = st[1], qe = st[2], sell = st[3];
    float init_price = bitf(st[0]);
    i32 qsum = 0;
    for (int i = 0; i < nT; ++i) {
        const i32* r = tr + i * 8;
        if (r[0] >= 0 && (r[6] == tid || r[7] == tid)) qsum = wadd(qsum, r[1]);
    }
    i32 qets = iabs(qsum);
    i32 quant_left = wsub(task, wadd(qe, qets));
    i32 pen = wmul(tc->doom_price_penalty, tick);
    float mids[HFTLOB_MAX_MSGS];
    for (int m = 0; m < M; ++m) mids[m] = i2f(wadd(bbb[m * 2], bba[m * 2])) / 2.0f;
    float avg_mid = wsum(mids, M) / (float)M;
    i32 side_sign = wsub(wmul(sell, 2), 1);
    i32 refp;
    /* a non-integer doom_price_penalty is a Python float: the far-touch price is then f32 */
    float penf = tc->doom_penalty_is_float ? tc->doom_penalty_f32 : i2f(pen);
    if (tc->reference_price == HFTLOB_PRICE_FAR_TOUCH && !tc->doom_penalty_is_float)
        refp = sell ? wmul(ifloordiv(wsub(bbb[(M - 1) * 2], pen), tick), tick)
                    : wmul(ifloordiv(wadd(bba[(M - 1) * 2], pen), tick), tick);
    else if (tc->reference_price == HFTLOB_PRICE_FAR_TOUCH)
        refp = sell ? f2i(ffloordiv(i2f(bbb[(M - 1) * 2]) - penf, (float)tick) * (float)tick)
                    : f2i(ffloordiv(i2f(bba[(M - 1) * 2]) + penf, (float)tick) * (float)tick);
    else
        refp = sell ? f2i(ffloordiv(avg_mid - penf, (float)tick) * (float)tick)
                    : f2i(ffloordiv(avg_mid + penf, (float)tick) * (float)tick);
    if (ep_done && quant_left > 0) {
        i32 row[8] = {refp, wmul(side_sign, iabs(quant_left)), c->artificial_order_id, c->placeholder_order_id,
                      0, 0, c->artificial_trader_id, tid};
        add_trade(tr, nT, row);
    }
    R->doom_quant = wmul(ep_done, quant_left);
    i32 aq = 0, oq = 0, qp = 0;
    float dur[HFTLOB_MAX_SLOTS], vw[HFTLOB_MAX_SLOTS];
    i32 init0 = LOADED(E)[0];
    for (int i = 0; i < nT; ++i) {
        const i32* r = tr + i * 8;
        int valid = r[0] >= 0;
        int mine = valid && (tid == r[6] || tid == r[7]);
        i32 P = valid ? r[0] : 0, Q = valid ? r[1] : 0, S = valid ? r[4] : 0;
        if (mine) {
            aq = wadd(aq, iabs(Q));
            qp = wadd(qp, wmul(ifloordiv(P, tick), iabs(Q)));
            dur[i] = i2f(iabs(Q)) / i2f(task) * i2f(wsub(S, init0));
        } else {
            oq = wadd(oq, iabs(Q));
            dur[i] = i2f(0) / i2f(task) * i2f(wsub(0, init0));
        }
    }
    float pv;
    if (oq == 0) pv = ffloordiv(avg_mid, (float)tick);
    else {
        for (int i = 0; i < nT; ++i) {
            const i32* r = tr + i * 8;
            int valid = r[0] >= 0;
            int mine = valid && (tid == r[6] || tid == r[7]);
            i32 P = (valid && !mine) ? r[0] : 0, Q = (valid && !mine) ? r[1] : 0;
            vw[i] = i2f(ifloordiv(P, tick)) * (i2f(iabs(Q)) / i2f(oq));
        }
        pv = wsum(vw, nT);
    }
    i32 dirs = isign(wsub(wmul(sell, 2), 1));
    float adv = i2f(dirs) * (i2f(qp) - pv * i2f(aq));
    float drift = i2f(wmul(dirs, aq)) * (pv - ffloordiv(init_price, (float)tick));
    float padv = adv / (i2f(aq) + 1e-9f);
    float pdrift = drift / (i2f(aq) + 1e-9f);
    float slip = adv + drift;
    i32 sc = LOADED(E)[5];
    float scf = i2f(sc), sc1 = i2f(wadd(sc, 1));
    R->vwap_rm = (bitf(st[11]) * scf + pv) / sc1;
    R->price_adv_rm = (bitf(st[9]) * scf + padv) / sc1;
    R->slippage_rm = (bitf(st[8]) * scf + slip) / sc1;
    R->price_drift_rm = (bitf(st[10]) * scf + pdrift) / sc1;
    float reward = adv + tc->reward_lambda * drift;
    R->trade_duration = bitf(st[12]) + wsum(dur, nT);
    R->quant_left = wsub(wsub(task, qe), aq);
    R->reward_info = reward; /* info["reward"] is taken before the finish_fast override */
    if (tc->reward_function == HFTLOB_EXE_REW_FINISH_FAST) reward = i2f(wsub(0, iabs(R->quant_left)));
    if (tc->reward_function == HFTLOB_EXE_REW_SIMPLEST_CASE) { /* exec_env.py:1723-1731 */
        float ps[HFTLOB_MAX_SLOTS];
        for (int i = 0; i < nT; ++i) {
            const i32* r = tr + i * 8;
            int valid = r[0] >= 0;
            int mine = valid && (tid == r[6] || tid == r[7]);
            /* agentTrades rows are 0 outside the agent's executed trades: price_slip = 0 - init_price there */
            float slip = i2f(mine ? r[0] : 0) - init_price;
            ps[i] = (sell ? slip : -slip) * i2f(mine ? iabs(r[1]) : 0);
        }
        reward = wsum(ps, nT);
    }
    R->reward = reward;
    R->p_vwap = pv;
    R->advantage = adv;
    R->drift = drift;
    R->slippage = slip;
    R->agentQuant = aq;
    R->qp_agent = qp;
}

/* ---- observations */
static float nrm(float x, float s, int norm) { return norm ? x / s : x; }

/* MM _get_obs_basic / _get_obs_engineered (fixed_steps) — mm_env.py:2963-3154 */
static void mm_obs(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st, float* o) {
    int M = c->n_msgs, nO = c->lob.n_orders, nz = tc->normalize;
    i32 pa = BASKS(E)[(M - 1) * 2], pb = BBIDS(E)[(M - 1) * 2];
    i32 spread = iabs(wsub(pa, pb));
    if (tc->observation_space == HFTLOB_MM_OBS_BASIC) { /* sorted keys: inventory, spread */
        o[0] = nrm(i2f(st[2]), 10.0f, nz);
        o[1] = nrm(i2f(spread), 1e4f, nz);
        return;
    }
    if (tc->observation_space == HFTLOB_MM_OBS_MESSAGES) return; /* the obs is the message array (msgs_out) */
    if (c->ep_type == 1) { /* mm_env.py:3029-3088: 10 sorted keys */
        const i32* W = WORLD(E);
        const i32* L = LOADED(E);
        float tm = i2f(W[0]) + i2f(W[1]) / 1e9f;
        float time_elapsed = tm - (i2f(L[0]) + i2f(L[1]) / 1e9f);
        float time_remaining = (float)c->episode_time - time_elapsed;
        float v[10] = {bitf(W[4]), i2f(st[2]), bitf(W[3]), i2f(pa), i2f(pb), i2f(side_volume(ASKS(E), nO)),
                       i2f(side_volume(BIDS(E), nO)), i2f(spread), i2f(L[5]), time_remaining};
        float sd[10] = {10.0f, 10.0f, 1e6f, 1e6f, 1e6f, 1000.0f, 1000.0f, 1e4f, 10.0f, (float)c->episode_time};
        for (int k = 0; k < 10; ++k) o[k] = nrm(v[k], sd[k], nz);
        return;
    }
    /* inventory, mid_price, p_ask, p_bid, q_ask, q_bid, spread, step_counter */
    o[0] = nrm(i2f(st[2]), 10.0f, nz);
    o[1] = nrm(bitf(WORLD(E)[3]), 1e6f, nz);
    o[2] = nrm(i2f(pa), 1e6f, nz);
    o[3] = nrm(i2f(pb), 1e6f, nz);
    o[4] = nrm(i2f(side_volume(ASKS(E), nO)), 1000.0f, nz);
    o[5] = nrm(i2f(side_volume(BIDS(E), nO)), 1000.0f, nz);
    o[6] = nrm(i2f(spread), 1e4f, nz);
    o[7] = nrm(i2f(LOADED(E)[5]), 10.0f, nz);
}

/* EXE _get_obs — exec_env.py:1913-2079; sorted keys (fixed_steps 12, fixed_time 15) */
static void exe_obs(const hftlob_env_cfg* c, const hftlob_agent_type_cfg* tc, Env* E, const i32* st, float* o) {
    int M = c->n_msgs, nO = c->lob.n_orders, nz = tc->normalize;
    if (tc->observation_space == HFTLOB_EXE_OBS_BASIC) {
        /* _get_obs_basic :1879-1911; sorted keys best_ask_price, best_bid_price, remaining_quant */
        i32 a = BASKS(E)[(M - 1) * 2], b = BBIDS(E)[(M - 1) * 2], rq = wsub(st[1], st[2]);
        if (nz) {
            o[0] = i2f(wsub(a, 1550000)) / 1e3f;
            o[1] = i2f(wsub(b, 1550000)) / 1e3f;
            o[2] = i2f(rq) / (float)tc->task_size;
        } else {
            o[0] = i2f(a); o[1] = i2f(b); o[2] = i2f(rq);
        }
        return;
    }
    if (tc->observation_space == HFTLOB_EXE_OBS_SIMPLEST_CASE) {
        /* _get_obs_simplest_case :1841-1877; sorted keys mid_price, percent_remaining_quant,
         * percent_time_remaining */
        const i32* W = WORLD(E);
        const i32* L = LOADED(E);
        i32 tu0 = wsub(W[0], L[0]), tu1 = wsub(W[1], L[1]);
        float ep = (float)c->episode_time;
        float ptr = (ep - (i2f(tu0) + i2f(tu1) / 1e9f)) / ep;
        float prq = i2f(wsub(st[1], st[2])) / i2f(st[1]);
        float mid = bitf(W[3]);
        if (nz) {
            o[0] = (mid - 7560000.0f) / 1e3f;
            o[1] = (prq - 0.5f) / 1.0f;
            o[2] = (ptr - 0.5f) / 1.0f;
        } else {
            o[0] = mid; o[1] = prq; o[2] = ptr;
        }
        return;
    }
    i32 sell = st[3];
    i32 pa = BASKS(E)[(M - 1) * 2], pb = BBIDS(E)[(M - 1) * 2];
    i32 p_aggr = sell ? pb : pa, p_pass = sell ? pa : pb;
    i32 vb = side_volume(BIDS(E), nO), va = side_volume(ASKS(E), nO);
    i32 q_aggr = sell ? vb : va, q_pass = sell ? va : vb;
    float ip = bitf(st[0]);
    float ts = (float)tc->task_size;
    i32 ms = LOADED(E)[3], sc = LOADED(E)[5];
    float rr = ms == 0 ? 0.0f : 1.0f - i2f(sc) / i2f(ms);
    if (c->ep_type == 1) {
        /* fixed_time (exec_env.py:1940-2010), 15 sorted keys: delta_time, executed_quant, init_price,
         * is_sell_task, p_aggr, p_pass, q_aggr, q_pass, remaining_quant, remaining_ratio, spread,
         * step_counter, task_size, time, time_remaining.  time = t[0] + t[1]/1e9 (f32). */
        const i32* W = WORLD(E);
        const i32* L = LOADED(E);
        float tm = i2f(W[0]) + i2f(W[1]) / 1e9f;
        float te = tm - (i2f(L[0]) + i2f(L[1]) / 1e9f);
        float trem = (float)c->episode_time - te;
        float dt = bitf(W[4]);
        float v[15] = {dt, i2f(st[2]), ip, i2f(sell), i2f(p_aggr), i2f(p_pass), i2f(q_aggr), i2f(q_pass),
                       i2f(wsub(st[1], st[2])), rr, i2f(iabs(wsub(p_aggr, p_pass))), i2f(sc), i2f(st[1]), tm, trem};
        if (nz) {
            o[0] = dt / 10.0f;
            o[1] = i2f(st[2]) / ts;
            o[2] = ip / 1e7f;
            o[3] = i2f(sell) / 1.0f;
            o[4] = (i2f(p_aggr) - ip) / 1e5f;
            o[5] = (i2f(p_pass) - ip) / 1e5f;
            o[6] = i2f(q_aggr) / 1000.0f;
            o[7] = i2f(q_pass) / 1000.0f;
            o[8] = i2f(wsub(st[1], st[2])) / ts;
            o[9] = rr / 1.0f;
            o[10] = i2f(iabs(wsub(p_aggr, p_pass))) / 1e4f;
            o[11] = i2f(sc) / 30.0f;
            o[12] = i2f(st[1]) / ts;
            o[13] = tm / 1e5f;
            o[14] = trem / (float)c->episode_time;
        } else {
            for (int k = 0; k < 15; ++k) o[k] = v[k];
        }
        return;
    }
    if (nz) {
        o[0] = i2f(st[2]) / ts;
        o[1] = ip / 1e7f;
        o[2] = i2f(sell) / 1.0f;
        o[3] = (i2f(p_aggr) - ip) / 1e5f;
        o[4] = (i2f(p_pass) - ip) / 1e5f;
        o[5] = i2f(q_aggr) / 1000.0f;
        o[6] = i2f(q_pass) / 1000.0f;
        o[7] = i2f(wsub(st[1], st[2])) / ts;
        o[8] = rr / 1.0f;
        o[9] = i2f(iabs(wsub(p_aggr, p_pass))) / 1e4f;
        o[10] = i2f(sc) / 30.0f;
        o[11] = i2f(st[1]) / ts;
    } else {
        o[0] = i2f(st[2]); o[1] = ip; o[2] = i2f(sell); o[3] = i2f(p_aggr); o[4] = i2f(p_pass);
        o[5] = i2f(q_aggr); o[6] = i2f(q_pass); o[7] = i2f(wsub(st[1], st[2])); o[8] = rr;
        o[9] = i2f(iabs(wsub(p_aggr, p_pass))); o[10] = i2f(sc); o[11] = i2f(st[1]);
    }
}

/* get_observation(normalize=False, flatten=False) — the dict of save_raw_observations
 * (marl_env.py:684-685), written in sorted-key order as 32-bit words: int32 fields as
 * int32, float32 fields as their bits (mm_env.py:2963-3088, exec_env.py:1841-2079).
 * Restated from the reference dicts, not from the normalised path above. */
static void agent_obs_raw(const hftlob_env_cfg* c, int t, Env* E, const i32* st, i32* o) {
    const hftlob_agent_type_cfg* tc = &c->types[t];
    int M = c->n_msgs, nO = c->lob.n_orders, n = 0;
    const i32* W = WORLD(E);
    const i32* L = LOADED(E);
    i32 pa = BASKS(E)[(M - 1) * 2], pb = BBIDS(E)[(M - 1) * 2];
    i32 va = side_volume(ASKS(E), nO), vb = side_volume(BIDS(E), nO);
    float tm = i2f(W[0]) + i2f(W[1]) / 1e9f;
    float time_remaining = (float)c->episode_time - (tm - (i2f(L[0]) + i2f(L[1]) / 1e9f));
    for (int k = 0; k < c->obs_stride; ++k) o[k] = 0;
#define PI(x) (o[n++] = (x))
#define PF(x) (o[n++] = fbit(x))
    if (tc->kind == HFTLOB_AGENT_MM) {
        i32 spread = iabs(wsub(pa, pb));
        if (tc->observation_space == HFTLOB_MM_OBS_BASIC) { PI(st[2]); PI(spread); return; }  /* inventory, spread */
        if (tc->observation_space == HFTLOB_MM_OBS_MESSAGES) return;
        if (c->ep_type == 1) PF(bitf(W[4]));                                   /* delta_time */
        PI(st[2]); PF(bitf(W[3])); PI(pa); PI(pb); PI(va); PI(vb); PI(spread); PI(L[5]);
        if (c->ep_type == 1) PF(time_remaining);
        return;
    }
    if (tc->observation_space == HFTLOB_EXE_OBS_BASIC) { PI(pa); PI(pb); PI(wsub(st[1], st[2])); return; }
    if (tc->observation_space == HFTLOB_EXE_OBS_SIMPLEST_CASE) {
        i32 tu0 = wsub(W[0], L[0]), tu1 = wsub(W[1], L[1]);
        float ep = (float)c->episode_time;
        PF(bitf(W[3]));                                          /* mid_price */
        PF(i2f(wsub(st[1], st[2])) / i2f(st[1]));                /* percent_remaining_quant */
        PF((ep - (i2f(tu0) + i2f(tu1) / 1e9f)) / ep);            /* percent_time_remaining */
        return;
    }
    i32 sell = st[3], p_aggr = sell ? pb : pa, p_pass = sell ? pa : pb;
    i32 ms = L[3], sc = L[5];
    if (c->ep_type == 1) PF(bitf(W[4]));                         /* delta_time */
    PI(st[2]); PF(bitf(st[0])); PI(sell); PI(p_aggr); PI(p_pass); PI(sell ? vb : va); PI(sell ? va : vb);
    PI(wsub(st[1], st[2])); PF(ms == 0 ? 0.0f : 1.0f - i2f(sc) / i2f(ms)); PI(iabs(wsub(p_aggr, p_pass)));
    PI(sc); PI(st[1]);
    if (c->ep_type == 1) { PF(tm); PF(time_remaining); }
#undef PI
#undef PF
}

static void agent_obs(const hftlob_env_cfg* c, int t, Env* E, const i32* st, float* o) {
    const hftlob_agent_type_cfg* tc = &c->types[t];
    for (int k = 0; k < c->obs_stride; ++k) o[k] = 0.0f;
    if (tc->kind == HFTLOB_AGENT_MM) mm_obs(c, tc, E, st, o);
    else exe_obs(c, tc, E, st, o);
}

/* ---- reset: MARLEnv.reset_env — marl_env.py:129-207, BaseLOBEnv.reset_env base_env.py:218-234 */
static void env_reset_one(const hftlob_env_cfg* c, const u32* key, const i32* init_states, i32* rec, float* obs) {
    Env E = {c, rec};
    int part = c->prng_partitionable, nT = c->n_types;
    u32 keys[HFTLOB_MAX_TYPES + 1][2];
    for (int j = 0; j <= nT; ++j) oracle_split(key, nT + 1, j, part, keys[j]);
    i32 idx = c->window_selector == -1 ? oracle_randint(keys[nT], 0, c->n_windows, part) : c->window_selector;
    if (idx < 0) idx = 0; /* gather index clamps (XLA) */
    if (idx > c->n_windows - 1) idx = c->n_windows - 1;
    memcpy(rec, init_states + (size_t)idx * c->init_rec_words, (size_t)c->init_rec_words * sizeof(i32));
    i32 ba[2], bb[2];
    best_quotes(&c->lob, ASKS(&E), BIDS(&E), ba, bb);
    for (int m = 0; m < c->n_msgs; ++m) {
        BASKS(&E)[m * 2] = ba[0]; BASKS(&E)[m * 2 + 1] = ba[1];
        BBIDS(&E)[m * 2] = bb[0]; BBIDS(&E)[m * 2 + 1] = bb[1];
    }
    i32* w = WORLD(&E);
    float mid = i2f(wadd(bb[0], ba[0])) / 2.0f;
    w[0] = LOADED(&E)[0]; w[1] = LOADED(&E)[1];
    w[2] = c->order_id_counter_start;
    w[3] = fbit(mid);
    w[4] = fbit(0.0f);
    i32* st = rec + c->off_agents;
    int a = 0;
    for (int t = 0; t < nT; ++t) {
        const hftlob_agent_type_cfg* tc = &c->types[t];
        i32 sell = tc->task == HFTLOB_TASK_SELL ? 1 : 0;
        if (tc->kind == HFTLOB_AGENT_EXE && tc->task == HFTLOB_TASK_RANDOM) sell = oracle_randint(keys[t], 0, 2, part);
        for (int i = 0; i < tc->n_agents; ++i, ++a) {
            if (tc->kind == HFTLOB_AGENT_MM) {
                st[0] = 0; st[1] = 0; st[2] = 0; st[3] = fbit(0.0f); st[4] = fbit(0.0f);
            } else {
                st[0] = fbit(mid); st[1] = tc->task_size; st[2] = 0; st[3] = sell;
                st[4] = fbit(mid / (float)c->tick_size);
                for (int k = 5; k < 13; ++k) st[k] = fbit(0.0f);
            }
            if (obs) agent_obs(c, t, &E, st, obs + (size_t)a * c->obs_stride);
            st += agent_words(tc);
        }
    }
}

static int env_cfg_ok(const hftlob_env_cfg* c) {
    if (!lob_cfg_ok(&c->lob)) return 0;
    if ((c->ep_type != 0 && c->ep_type != 1) || c->n_types < 1 || c->n_types > HFTLOB_MAX_TYPES) return 0;
    if (c->n_msgs > HFTLOB_MAX_MSGS || c->n_agents > HFTLOB_MAX_AGENTS || c->n_windows < 1) return 0;
    if (c->obs_stride > HFTLOB_MAX_OBS) return 0;
    int words = 0;
    for (int t = 0; t < c->n_types; ++t) {
        const hftlob_agent_type_cfg* tc = &c->types[t];
        if (tc->kind == HFTLOB_AGENT_EXE && tc->action_space == HFTLOB_EXE_ACT_FIXED_PRICES &&
            (tc->n_actions < 1 || tc->n_actions > 4 || tc->action_width != tc->n_actions))
            return 0;
        words += tc->n_agents * tc->action_width;
    }
    return words == c->action_words;
}

int oracle_env_reset(const hftlob_env_cfg* c, int n_env, const u32* keys, const i32* init_states, i32* state,
                     float* obs) {
    if (!env_cfg_ok(c)) return HFTLOB_EINVAL;
#pragma omp parallel for schedule(dynamic, 16)
    for (int e = 0; e < n_env; ++e)
        env_reset_one(c, keys + 2 * e, init_states, state + (size_t)e * c->rec_words,
                      obs ? obs + (size_t)e * c->n_agents * c->obs_stride : NULL);
    return HFTLOB_OK;
}

/* ---- get_L2_state — JaxOrderBookArrays.py:1231-1264 (world debug_mode, marl_env.py:645-656).
 * bid levels: -unique(-bid_prices, size=n, fill_value=1) (an empty row's -1 is a level, the fill
 * reads -1), then -1 -> -maxint; ask levels: unique(where(p == -1, maxint, p), size=n,
 * fill_value=-1), then -1 -> maxint; volumes get_volume_at_price at the (replaced) level price,
 * negatives -> 0; out [n][4] = [ask_p, ask_q, bid_p, bid_q] (hstack((asks.T, bids.T)).flatten()). */
static int cmp_i32(const void* a, const void* b) {
    i32 x = *(const i32*)a, y = *(const i32*)b;
    return (x > y) - (x < y);
}
static void unique_sorted(i32* v, int n, int size, i32 fill, i32* out) {
    qsort(v, (size_t)n, sizeof(i32), cmp_i32);
    int k = 0;
    for (int i = 0; i < n && k < size; ++i)
        if (i == 0 || v[i] != v[i - 1]) out[k++] = v[i];
    for (; k < size; ++k) out[k] = fill;
}
static i32 volume_at(const i32* s, int nO, i32 p) {
    i32 v = 0;
    for (int i = 0; i < nO; ++i) if (s[i * 6] == p) v = wadd(v, s[i * 6 + 1]);
    return v;
}
int oracle_l2_state(const hftlob_lob_cfg* c, const i32* asks, const i32* bids, int n_levels, i32* out) {
    int nO = c->n_orders;
    i32 tmp[HFTLOB_MAX_SLOTS], lv[HFTLOB_MAX_SLOTS];
    /* the stack tables hold HFTLOB_MAX_SLOTS rows / levels (the env path refuses larger books) */
    if (nO < 1 || nO > HFTLOB_MAX_SLOTS || n_levels < 0 || n_levels > HFTLOB_MAX_SLOTS) return HFTLOB_ESHAPE;
    for (int i = 0; i < nO; ++i) tmp[i] = wmul(-1, bids[i * 6]);
    unique_sorted(tmp, nO, n_levels, 1, lv);
    for (int k = 0; k < n_levels; ++k) {
        i32 p = wmul(-1, lv[k]);
        p = p == -1 ? wsub(0, c->maxint) : p;
        i32 q = volume_at(bids, nO, p);
        out[k * 4 + 2] = p;
        out[k * 4 + 3] = q < 0 ? 0 : q;
    }
    for (int i = 0; i < nO; ++i) tmp[i] = asks[i * 6] == -1 ? c->maxint : asks[i * 6];
    unique_sorted(tmp, nO, n_levels, -1, lv);
    for (int k = 0; k < n_levels; ++k) {
        i32 p = lv[k] == -1 ? c->maxint : lv[k];
        i32 q = volume_at(asks, nO, p);
        out[k * 4] = p;
        out[k * 4 + 1] = q < 0 ? 0 : q;
    }
    return HFTLOB_OK;
}

/* ---- MARLEnv.step — marl_env.py:775-804 + step_env :211-709 */
static void env_step_one(const hftlob_env_cfg* c, const u32* key, const i32* act, const i32* msg_data,
                         const i32* init_states, i32* rec, float* obs, float* rew, i32* done_all, i32* dones,
                         i32* info, i32* obs_raw, i32* msgs_out, i32* debug) {
    Env E = {c, rec};
    int part = c->prng_partitionable, M = c->n_msgs, D = c->n_data_msg, A = c->n_action_msgs,
        C = c->n_cancel_msgs, nO = c->lob.n_orders, nT = c->lob.n_trades;
    u32 k1[2], key_reset[2], k2[2], shuffle_key[2];
    oracle_split(key, 2, 0, part, k1);
    oracle_split(key, 2, 1, part, key_reset);
    i32* L = LOADED(&E);
    i32* W = WORLD(&E);
    /* (B) data messages: dynamic_slice clamps the start into [0, N-D] */
    i32 start = wadd(L[4], wmul(D, L[5]));
    if (start < 0) start = 0;
    if (start > c->n_data_rows - D) start = c->n_data_rows - D;
    i32 comb[HFTLOB_MAX_MSGS * 8];
    memcpy(comb + (size_t)(C + A) * 8, msg_data + (size_t)start * 8, (size_t)D * 8 * sizeof(i32));
    if (c->ep_type == 1) { /* fixed_time: rows past init_time[0] + episode_time keep only their time (base_env.py:358-367) */
        i32 t_end = wadd(L[0], c->episode_time);
        for (int r = 0; r < D; ++r) {
            i32* row = comb + (size_t)(C + A + r) * 8;
            if (row[6] >= t_end) memset(row, 0, 6 * sizeof(i32));
        }
    }
    /* (C) agent messages */
    i32 actm[HFTLOB_MAX_MSGS * 8], cnlm[HFTLOB_MAX_MSGS * 8];
    ActX ax[HFTLOB_MAX_AGENTS];
    int na = 0, nc = 0, a = 0;
    const i32* av = act; /* agent a's action words (action_width of its type) */
    i32* st = rec + c->off_agents;
    i32* sts[HFTLOB_MAX_AGENTS];
    for (int t = 0; t < c->n_types; ++t) {
        const hftlob_agent_type_cfg* tc = &c->types[t];
        for (int i = 0; i < tc->n_agents; ++i, ++a) {
            sts[a] = st;
            i32 tid = wsub(tc->trader_id0, i);
            i32* am = actm + na * 8;
            i32* cm = cnlm + nc * 8;
            memset(&ax[a], 0, sizeof ax[a]);
            const i32* aa = av;
            av += tc->action_width;
            if (tc->kind == HFTLOB_AGENT_MM) {
                if (tc->action_space == HFTLOB_MM_ACT_DIRECTIONAL) mm_directional(c, tc, &E, tid, aa[0], am, &ax[a]);
                else if (tc->action_space == HFTLOB_MM_ACT_FIXED_QUANTS) mm_fixed_quant(c, tc, &E, st, tid, aa[0], am, &ax[a]);
                else mm_other_actions(c, tc, &E, st, tid, aa[0], am, &ax[a]);
                int sz = tc->n_msgs / 4;
                get_cancel_msgs(BIDS(&E), nO, tid, sz, 1, W[0], W[1], cm);
                get_cancel_msgs(ASKS(&E), nO, tid, sz, -1, W[0], W[1], cm + sz * 8);
            } else {
                if (tc->action_space == HFTLOB_EXE_ACT_FIXED_PRICES) exe_fixed_price(c, tc, &E, st, tid, aa, am);
                else exe_fqc(c, tc, &E, st, tid, aa[0], am);
                i32 sell = st[3];
                get_cancel_msgs(sell ? ASKS(&E) : BIDS(&E), nO, tid, tc->n_msgs / 2, wsub(1, wmul(sell, 2)), W[0], W[1],
                                cm);
            }
            filter_messages(am, cm, tc->n_action_msgs);
            na += tc->n_action_msgs;
            nc += tc->n_msgs - tc->n_action_msgs;
            st += agent_words(tc);
        }
    }
    /* order ids: counter, counter-1, ... ; then shuffle (permutation of rows) */
    i32 ctr = W[2];
    for (int j = 0; j < A; ++j) actm[j * 8 + 4] = wsub(ctr, j);
    i32 new_ctr = wsub(ctr, A);
    int perm[HFTLOB_MAX_MSGS];
    for (int j = 0; j < A; ++j) perm[j] = j;
    const u32* scan_key = k1; /* marl_env.py:293-294: key, shuffle_key = split(key); scan(key) :349-351 */
    if (c->shuffle_action_messages) {
        oracle_split(k1, 2, 0, part, k2);
        oracle_split(k1, 2, 1, part, shuffle_key);
        oracle_permutation(shuffle_key, A, part, perm);
        scan_key = k2;
    }
    memcpy(comb, cnlm, (size_t)C * 8 * sizeof(i32));
    for (int j = 0; j < A; ++j) memcpy(comb + (size_t)(C + j) * 8, actm + (size_t)perm[j] * 8, 8 * sizeof(i32));
    if (msgs_out) memcpy(msgs_out, comb, (size_t)M * 8 * sizeof(i32)); /* the "messages" observation */
    /* (D) book: trades reinitialised to -1, then the scan */
    i32 asks[HFTLOB_MAX_SLOTS * 6], bids[HFTLOB_MAX_SLOTS * 6], trades[HFTLOB_MAX_SLOTS * 8];
    memcpy(asks, ASKS(&E), (size_t)nO * 6 * sizeof(i32));
    memcpy(bids, BIDS(&E), (size_t)nO * 6 * sizeof(i32));
    for (int i = 0; i < nT * 8; ++i) trades[i] = -1;
    i32 bba[HFTLOB_MAX_MSGS * 2], bbb[HFTLOB_MAX_MSGS * 2];
    for (int m = 0; m < M; ++m) {
        process_msg(&c->lob, comb + m * 8, asks, bids, trades, scan_key, M, m);
        best_quotes(&c->lob, asks, bids, bba + m * 2, bbb + m * 2);
    }
    int abort_ep = 0;
    for (int m = 0; m < M; ++m) abort_ep |= (bba[m * 2] == -1) || (bbb[m * 2] == -1);
    /* _ffill_best_prices — marl_env.py:723-749 */
    i32* old_ba = BASKS(&E);
    i32* old_bb = BBIDS(&E);
    for (int side = 0; side < 2; ++side) {
        i32* pq = side ? bbb : bba;
        i32 last = side ? old_bb[(M - 1) * 2] : old_ba[(M - 1) * 2];
        if (pq[0] == -1) { pq[0] = last; pq[1] = 0; }
        for (int m = 0; m < M; ++m) if (pq[m * 2] == -1) pq[m * 2 + 1] = 0;
        i32 prev = -1;
        for (int m = 0; m < M; ++m) { if (pq[m * 2] != -1) prev = pq[m * 2]; pq[m * 2] = prev; }
    }
    i32 ft0 = comb[(M - 1) * 8 + 6], ft1 = comb[(M - 1) * 8 + 7];
    int ep_done = wsub(wsub(L[3], L[5]), 1) <= 1;
    /* (E) rewards against the OLD world state */
    MMRew mr[HFTLOB_MAX_AGENTS];
    EXRew er[HFTLOB_MAX_AGENTS];
    a = 0;
    for (int t = 0; t < c->n_types; ++t) {
        const hftlob_agent_type_cfg* tc = &c->types[t];
        for (int i = 0; i < tc->n_agents; ++i, ++a) {
            i32 tid = wsub(tc->trader_id0, i);
            if (tc->kind == HFTLOB_AGENT_MM) mm_reward(c, tc, &E, sts[a], tid, trades, bba, bbb, ep_done, &mr[a]);
            else exe_reward(c, tc, &E, sts[a], tid, trades, bba, bbb, ep_done, &er[a]);
        }
    }
    /* (F) world update */
    float old_mid = bitf(W[3]);
    (void)old_mid;
    i32 ot0 = W[0], ot1 = W[1];
    if (debug) { /* world debug_mode: lob_state of the stepped books, then the step's trades */
        oracle_l2_state(&c->lob, asks, bids, HFTLOB_L2_LEVELS, debug);
        memcpy(debug + 4 * HFTLOB_L2_LEVELS, trades, (size_t)nT * 8 * sizeof(i32));
    }
    memcpy(ASKS(&E), asks, (size_t)nO * 6 * sizeof(i32));
    memcpy(BIDS(&E), bids, (size_t)nO * 6 * sizeof(i32));
    memcpy(TRADES(&E), trades, (size_t)nT * 8 * sizeof(i32));
    memcpy(BASKS(&E), bba, (size_t)M * 2 * sizeof(i32));
    memcpy(BBIDS(&E), bbb, (size_t)M * 2 * sizeof(i32));
    L[5] = wadd(L[5], 1);
    float new_mid = i2f(wadd(bbb[(M - 1) * 2], bba[(M - 1) * 2])) / 2.0f;
    float dt = i2f(ft0) + i2f(ft1) / 1e9f - i2f(ot0) - i2f(ot1) / 1e9f;
    W[0] = ft0; W[1] = ft1; W[2] = new_ctr; W[3] = fbit(new_mid); W[4] = fbit(dt);
    /* (G) agent state update + dones; (K) observations */
    int all = ep_done;
    *done_all = all;
    a = 0;
    for (int t = 0; t < c->n_types; ++t) {
        const hftlob_agent_type_cfg* tc = &c->types[t];
        for (int i = 0; i < tc->n_agents; ++i, ++a) {
            i32* s = sts[a];
            int d = 0;
            i32* ai = info ? info + HFTLOB_INFO_WORLD_WORDS + a * HFTLOB_INFO_AGENT_WORDS : NULL;
            if (tc->kind == HFTLOB_AGENT_MM) {
                s[0] = ax[a].bid_dist; s[1] = ax[a].ask_dist; s[2] = mr[a].end_inventory;
                s[3] = fbit(bitf(s[3]) + mr[a].PnL); s[4] = fbit(mr[a].cash);
                d = 0;
                rew[a] = mr[a].reward / tc->reward_scaling_quo;
                if (ai) {
                    const MMRew* R = &mr[a];
                    float fl[] = {R->reward, R->reward_pv, R->reward_spooner, R->end_of_ep_pv,
                                  R->reward_spooner_damped, R->reward_spooner_asym_damped,
                                  R->reward_spooner_asym_damped2, R->reward_delta_pv, bitf(s[3])};
                    for (int k = 0; k < 9; ++k) ai[k] = fbit(fl[k]);
                    ai[9] = d; ai[10] = s[2]; ai[11] = fbit(R->delta_mid); ai[12] = fbit(R->market_share);
                    ai[13] = fbit(R->buyPnL); ai[14] = R->forced_unwind; ai[15] = fbit(R->invPnL);
                    ai[16] = ax[a].bid_price; ai[17] = ax[a].ask_price; ai[18] = ax[a].bid_dist;
                    ai[19] = ax[a].ask_dist; ai[20] = ax[a].ask_quant; ai[21] = ax[a].bid_quant;
                    ai[22] = fbit(R->sellPnL); ai[23] = fbit(R->inventoryValue);
                }
            } else {
                const EXRew* R = &er[a];
                s[2] = wadd(s[2], R->agentQuant);
                s[4] = fbit(R->p_vwap);
                s[5] = fbit(bitf(s[5]) + i2f(R->qp_agent));
                s[6] = fbit(bitf(s[6]) + R->drift);
                s[7] = fbit(bitf(s[7]) + R->advantage);
                s[8] = fbit(R->slippage_rm); s[9] = fbit(R->price_adv_rm); s[10] = fbit(R->price_drift_rm);
                s[11] = fbit(R->vwap_rm); s[12] = fbit(R->trade_duration);
                d = wsub(s[1], s[2]) <= 0;
                rew[a] = R->reward / tc->reward_scaling_quo;
                if (ai) {
                    memset(ai, 0, HFTLOB_INFO_AGENT_WORDS * sizeof(i32));
                    ai[0] = R->quant_left; ai[1] = d; ai[2] = fbit(R->slippage); ai[3] = fbit(R->vwap_rm);
                    ai[4] = fbit(R->drift); ai[5] = fbit(R->advantage); ai[6] = R->doom_quant; ai[7] = s[3];
                    ai[8] = fbit(R->reward_info);
                }
            }
            dones[a] = d;
            float* o = obs + (size_t)a * c->obs_stride;
            agent_obs(c, t, &E, s, o);
            if (obs_raw) agent_obs_raw(c, t, &E, s, obs_raw + (size_t)a * c->obs_stride);
            if (d && !all) for (int k = 0; k < c->obs_stride; ++k) o[k] = 0.0f;
        }
    }
    if (info) {
        float sa[HFTLOB_MAX_MSGS], sb[HFTLOB_MAX_MSGS];
        for (int m = 0; m < M; ++m) { sa[m] = i2f(bba[m * 2]); sb[m] = i2f(bbb[m * 2]); }
        info[0] = L[2]; info[1] = W[3]; info[2] = L[5]; info[3] = W[0]; info[4] = W[1]; info[5] = W[2];
        info[6] = bba[(M - 1) * 2]; info[7] = bbb[(M - 1) * 2];
        info[8] = fbit(wsum(sa, M) / (float)M); info[9] = fbit(wsum(sb, M) / (float)M);
        info[10] = W[4]; info[11] = ep_done; info[12] = abort_ep;
        info[13] = wsub(bba[(M - 1) * 2], bbb[(M - 1) * 2]);
    }
    /* auto-reset: state and obs from reset(key_reset) when __all__ */
    if (all) env_reset_one(c, key_reset, init_states, rec, obs);
}

int oracle_env_step_dbg(const hftlob_env_cfg* c, int n_env, const u32* keys, const i32* actions, const i32* msg_data,
                        const i32* init_states, i32* state, float* obs, float* rew, i32* done_all, i32* dones,
                        i32* info, i32* obs_raw, i32* msgs, i32* debug) {
    if (!env_cfg_ok(c)) return HFTLOB_EINVAL;
    const size_t dw = (size_t)HFTLOB_DEBUG_WORDS(c->lob.n_trades);
#pragma omp parallel for schedule(dynamic, 16)
    for (int e = 0; e < n_env; ++e)
        env_step_one(c, keys + 2 * e, actions + (size_t)e * c->action_words, msg_data, init_states,
                     state + (size_t)e * c->rec_words, obs + (size_t)e * c->n_agents * c->obs_stride,
                     rew + (size_t)e * c->n_agents, done_all + e, dones + (size_t)e * c->n_agents,
                     info ? info + (size_t)e * c->info_words : NULL,
                     obs_raw ? obs_raw + (size_t)e * c->n_agents * c->obs_stride : NULL,
                     msgs ? msgs + (size_t)e * c->n_msgs * 8 : NULL, debug ? debug + (size_t)e * dw : NULL);
    return HFTLOB_OK;
}
int oracle_env_step_ex(const hftlob_env_cfg* c, int n_env, const u32* keys, const i32* actions, const i32* msg_data,
                       const i32* init_states, i32* state, float* obs, float* rew, i32* done_all, i32* dones,
                       i32* info, i32* obs_raw, i32* msgs) {
    return oracle_env_step_dbg(c, n_env, keys, actions, msg_data, init_states, state, obs, rew, done_all, dones, info,
                               obs_raw, msgs, NULL);
}
int oracle_env_step(const hftlob_env_cfg* c, int n_env, const u32* keys, const i32* actions, const i32* msg_data,
                    const i32* init_states, i32* state, float* obs, float* rew, i32* done_all, i32* dones,
                    i32* info) {
    return oracle_env_step_ex(c, n_env, keys, actions, msg_data, init_states, state, obs, rew, done_all, dones, info,
                              NULL, NULL);
}

/* Speed_test.py:166-177 action sampling */
void oracle_sample_actions(const hftlob_env_cfg* c, int n_env, const u32* keys, i32* actions) {
    int part = c->prng_partitionable;
    for (int e = 0; e < n_env; ++e) {
        i32* out = actions + (size_t)e * c->action_words;
        for (int t = 0; t < c->n_types; ++t) {
            const hftlob_agent_type_cfg* tc = &c->types[t];
            u32 sub[2];
            oracle_split(keys + 2 * e, c->n_types, t, part, sub);
            for (int i = 0; i < tc->n_agents; ++i) {
                u32 ki[2];
                oracle_split(sub, tc->n_agents, i, part, ki);
                if (tc->kind == HFTLOB_AGENT_EXE && tc->action_space == HFTLOB_EXE_ACT_FIXED_PRICES) {
                    /* MultiDiscrete([fixed_quant_value] * n_actions).sample (spaces.py:57-65) */
                    for (int j = 0; j < tc->n_actions; ++j)
                        *out++ = randint_shaped(ki, tc->n_actions, j, 0, tc->fixed_quant_value, part);
                } else {
                    *out++ = oracle_randint(ki, 0, tc->n_actions, part); /* Discrete.sample */
                }
            }
        }
    }
}

void oracle_split_keys(int n_env, int n, int part, const u32* keys, u32* out) {
    for (int e = 0; e < n_env; ++e)
        for (int j = 0; j < n; ++j) oracle_split(keys + 2 * e, n, j, part, out + ((size_t)e * n + j) * 2);
}

/* One MM agent's raw action messages (before _filter_messages) for the env
 * record `rec`: the agent-level checker of the action spaces (tests only).
 * out: 2 rows of 8; extras: bid_price, ask_price, bid_dist, ask_dist, bid_quant,
 * ask_quant, empty_book. */
int oracle_mm_action_msgs(const hftlob_env_cfg* c, int type, int agent, const i32* rec, const i32* action_words,
                          i32* out, i32* extras) {
    i32 action = action_words[0];
    if (type < 0 || type >= c->n_types) return HFTLOB_EINVAL;
    if (c->types[type].kind == HFTLOB_AGENT_EXE) { /* EXE: up to 4 rows, no extras */
        const hftlob_agent_type_cfg* te = &c->types[type];
        int off = c->off_agents;
        for (int t = 0; t < type; ++t) off += c->types[t].n_agents * agent_words(&c->types[t]);
        Env E = {c, (i32*)rec};
        const i32* st = rec + off + agent * agent_words(te);
        if (te->action_space == HFTLOB_EXE_ACT_FIXED_PRICES)
            exe_fixed_price(c, te, &E, st, wsub(te->trader_id0, agent), action_words, out);
        else
            exe_fqc(c, te, &E, st, wsub(te->trader_id0, agent), action, out);
        memset(extras, 0, 7 * sizeof(i32));
        return HFTLOB_OK;
    }
    const hftlob_agent_type_cfg* tc = &c->types[type];
    Env E = {c, (i32*)rec};
    int a0 = 0, off = c->off_agents;
    for (int t = 0; t < type; ++t) {
        a0 += c->types[t].n_agents;
        off += c->types[t].n_agents * agent_words(&c->types[t]);
    }
    const i32* st = rec + off + agent * agent_words(tc);
    i32 tid = wsub(tc->trader_id0, agent);
    ActX x;
    memset(&x, 0, sizeof x);
    if (tc->action_space == HFTLOB_MM_ACT_DIRECTIONAL) mm_directional(c, tc, &E, tid, action, out, &x);
    else if (tc->action_space == HFTLOB_MM_ACT_FIXED_QUANTS) mm_fixed_quant(c, tc, &E, st, tid, action, out, &x);
    else mm_other_actions(c, tc, &E, st, tid, action, out, &x);
    i32 ex[7] = {x.bid_price, x.ask_price, x.bid_dist, x.ask_dist, x.bid_quant, x.ask_quant, x.empty_book};
    memcpy(extras, ex, sizeof ex);
    (void)a0;
    return HFTLOB_OK;
}

/* struct layout of include/hftlob.h as the C compiler sees it (ABI test) */
#include <stddef.h>
void oracle_abi_layout(int* out) {
    out[0] = (int)sizeof(hftlob_lob_cfg);
    out[1] = (int)sizeof(hftlob_agent_type_cfg);
    out[2] = (int)sizeof(hftlob_env_cfg);
    out[3] = (int)offsetof(hftlob_env_cfg, types);
    out[4] = (int)offsetof(hftlob_agent_type_cfg, rebate_factor);
    out[5] = (int)sizeof(hftlob_step_out);
    out[6] = (int)offsetof(hftlob_env_cfg, info_words);
    out[7] = (int)offsetof(hftlob_agent_type_cfg, task);
}

#ifdef _OPENMP
#include <omp.h>
#endif
/* thread count of the OpenMP loops (CPU-baseline sizing); returns the value in effect */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* Speed_test's rollout (Speed_test.py:186-196) on the CPU, the loop in C:
 *   per step t: master, *step_keys = split(master, key_n + 1)
 *               env e (global index key_e0 + e): actions = Discrete.sample per agent
 *               (Speed_test.py:166-177), then MARLEnv.step with auto-reset.
 * The master-key chain is derived first; then every env runs all n_steps on one
 * thread (OpenMP over envs).  `master` [2] is advanced in place; `state` is
 * [n_env][rec_words], updated in place.  The CPU baseline of bench.py and the
 * metric-shape parity tests use it (test infrastructure, like the rest of this file). */
int oracle_rollout_sampled(const hftlob_env_cfg* c, int n_env, int key_e0, int key_n, int n_steps, u32* master,
                           const i32* msg_data, const i32* init_states, i32* state) {
    if (!env_cfg_ok(c) || n_env < 0 || n_steps < 0 || key_e0 < 0 || key_n < key_e0 + n_env) return HFTLOB_EINVAL;
    int part = c->prng_partitionable;
    u32* chain = (u32*)malloc(sizeof(u32) * 2 * (size_t)(n_steps + 1));
    if (!chain) return HFTLOB_EINVAL;
    chain[0] = master[0];
    chain[1] = master[1];
    for (int t = 0; t < n_steps; ++t) oracle_split(chain + 2 * t, key_n + 1, 0, part, chain + 2 * (t + 1));
#pragma omp parallel for schedule(dynamic, 4)
    for (int e = 0; e < n_env; ++e) {
        float obs[HFTLOB_MAX_AGENTS * HFTLOB_MAX_OBS], rew[HFTLOB_MAX_AGENTS];
        i32 dones[HFTLOB_MAX_AGENTS], acts[HFTLOB_MAX_AGENTS * 4], done_all;
        i32* rec = state + (size_t)e * c->rec_words;
        for (int t = 0; t < n_steps; ++t) {
            u32 key[2];
            oracle_split(chain + 2 * t, key_n + 1, key_e0 + e + 1, part, key);
            oracle_sample_actions(c, 1, key, acts);
            env_step_one(c, key, acts, msg_data, init_states, rec, obs, rew, &done_all, dones, NULL, NULL, NULL, NULL);
        }
    }
    master[0] = chain[2 * n_steps];
    master[1] = chain[2 * n_steps + 1];
    free(chain);
    return HFTLOB_OK;
}
