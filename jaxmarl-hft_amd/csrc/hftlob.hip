// hftlob.hip — MI355X (gfx950 / CDNA4) limit-order-book engine and fused
// multi-agent env step, behind the C ABI of include/hftlob.h.
//
// Execution model: ONE 64-lane wavefront per environment.  The book lives in
// LDS as structure-of-arrays tables (per side [6 fields][nO slots], trade log
// [8][nT]); slot s maps to lane s&63, register set s>>6 when a column is
// loaded.  The message stream is taken 64 rows at a time (row m -> lane m&63),
// decoded for the whole chunk in VALU, and each message is read into SGPRs
// with v_readlane, so the per-message dispatch is a wave-uniform scalar branch
// (only the taken handler runs — the XLA reference evaluates all five
// lax.switch branches under vmap).  Price-time priority, first-free-slot,
// best-quote and volume queries are DPP wave reductions and ballots.
// The CU's single scalar ALU, shared by its 16 resident waves, is the scarce
// resource: the code keeps per-lane work in VALU and uniform state in one
// flag word.
//
// Semantics follow the reference line by line (cited per function), including
// its quirks.  Integer state is bit-exact with the
// oracle; float32 arithmetic follows the jnp expression order, and float sums
// use the canonical wave order (fold lane l+64k, then xor butterfly 1..32).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <mutex>
#include <type_traits>
#include <limits.h>

#include "../../include/hftlob.h"

typedef int32_t i32;
typedef uint32_t u32;
typedef uint8_t u8;
#define DEV __device__ __forceinline__

// ---------------------------------------------------------------- wave utils
DEV int lane_id() { return __lane_id(); }
DEV i32 rdl(i32 v, int l) { return __builtin_amdgcn_readlane(v, l); }
DEV i32 wrl(i32 old, i32 val, int l) { return __lane_id() == l ? val : old; }  // v_cmp + v_cndmask
DEV i32 uni(i32 v) { return __builtin_amdgcn_readfirstlane(v); }
DEV float unif(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
DEV i32 wadd(i32 a, i32 b) { return (i32)((u32)a + (u32)b); }
DEV i32 wsub(i32 a, i32 b) { return (i32)((u32)a - (u32)b); }
DEV i32 wmul(i32 a, i32 b) { return (i32)((u32)a * (u32)b); }
DEV i32 iabs_(i32 a) { return a < 0 ? wsub(0, a) : a; }
DEV i32 isign(i32 a) { return (a > 0) - (a < 0); }
DEV i32 imax_(i32 a, i32 b) { return a > b ? a : b; }
DEV i32 imin_(i32 a, i32 b) { return a < b ? a : b; }
DEV float i2f(i32 a) { return (float)a; }
DEV i32 f2i(float f) { return (i32)f; }
DEV float bitf(i32 w) { return __int_as_float(w); }
DEV i32 fbit(float f) { return __float_as_int(f); }

// jnp.floor_divide for int32
DEV i32 ifloordiv(i32 a, i32 b) {
    i32 q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
    return q;
}
// jnp.floor_divide(a, tick_size), exactly, by a multiply: with l = ceil(log2 d) and
// m = ceil(2^(31+l) / d) < 2^32 (hftlob_env_cfg.tick_magic, set by the launch code),
// floor(n / d) = (n * m) >> (31 + l) for every 0 <= n < 2^31 (Granlund & Montgomery 1994, thm 4.2,
// N = 31); a negative a divides ~a = -a - 1 and the quotient's complement is the floor
// (tools/magic_check.c checks every int32 numerator for d = 1, 3, 100)
DEV i32 tick_floordiv(const hftlob_env_cfg& c, i32 a) {
    const u32 d = (u32)c.tick_size;
    const int sh = 31 + (d > 1u ? 32 - __builtin_clz(d - 1u) : 0);
    const u32 n = a < 0 ? ~(u32)a : (u32)a;
    const u32 q = (u32)(((unsigned long long)n * c.tick_magic) >> sh);
    return a < 0 ? (i32)~q : (i32)q;
}
// fmodf, exactly, without the library's bit-by-bit reduction loop when |x / y| < 2^23 (prices
// over a tick): with the correctly rounded quotient q' of |x| / |y| < 2^23, trunc(q') is the true
// quotient Q or Q + 1 (Q and Q + 1 are floats and rounding is monotonic), so |x| - trunc(q')|y|
// lies in [-|y|, |y|) and is a multiple of the smaller ulp: the fma computes it exactly, and adding
// |y| back to a negative one is exact too.  NaN, inf, zero and huge quotients take fmodf.
DEV float fmod_exact(float x, float y) {
    const float ax = fabsf(x), ay = fabsf(y), qf = ax / ay;
    if (!(qf < 8388608.0f) | !(ay > 0.0f) | !(ay < INFINITY)) return fmodf(x, y);
    float r = fmaf(-truncf(qf), ay, ax);
    r = r < 0.0f ? r + ay : r;
    return copysignf(r, x);
}
// jnp.floor_divide for float32 (jax _float_divmod, round half away from zero)
DEV float ffloordiv(float x, float y) {
    float mod = fmod_exact(x, y);
    float div = (x - mod) / y;
    bool ind = (mod != 0.0f) && (((y > 0) - (y < 0)) != ((mod > 0) - (mod < 0)));
    if (ind) div = div - 1.0f;
    return roundf(div);
}

// jnp.floor_divide(x, float(tick_size)) for float32 x: with y = tick_size an integer below 2^24
// and |x| < 2^24, ffloordiv returns floor(x / y) exactly (fmod_exact is exact, x - fmod(x, y) is
// y * trunc(x / y), an integer below 2^24, so the division is exact and the floor adjustment is
// the real floor; x = -0 gives +0).  Here, for a = |x|: k = floor(a * rcp(y)) is floor(a / y) or
// off by one (a / y < 2^19, rcp within 4 ulp), and the remainder r = a - k y is exact (a multiple
// of ulp(a), below y and no larger than a once corrected), so one correction step gives
// floor(a / y) and r; then floor(x / y) = -(floor(a / y) + (r != 0)) for x < 0.  Outside those
// bounds (and NaN / inf) it takes ffloordiv.  tools/ffloordiv_check.c checks it bit for bit
// against the jnp formula.
DEV float tick_ffloordiv(const hftlob_env_cfg& c, float x) {
    const float y = (float)c.tick_size, a = fabsf(x);
    const float q = a * __builtin_amdgcn_rcpf(y);
    if (!((a < 16777216.0f) & (q < 524288.0f) & (c.tick_size < (1 << 24)))) return ffloordiv(x, y);
    float k = floorf(q), r = fmaf(-k, y, a);
    if (r < 0.0f) { k -= 1.0f; r += y; }
    else if (r >= y) { k += 1.0f; r -= y; }
    return (x < 0.0f ? -(k + (r != 0.0f ? 1.0f : 0.0f)) : k) + 0.0f;
}

// DPP all-reduce across the wave; result is wave-uniform (SGPR).
// quad_perm[1,0,3,2], quad_perm[2,3,0,1], row_half_mirror, row_mirror,
// row_bcast:15 (rows 1,3), row_bcast:31 (rows 2,3) -> lane 63 holds the total.
#define DPPX(idv, v, ctrl, rmask) __builtin_amdgcn_update_dpp((idv), (v), (ctrl), (rmask), 0xF, false)
DEV i32 wave_max(i32 v) {
    v = imax_(v, DPPX(INT_MIN, v, 0xB1, 0xF));
    v = imax_(v, DPPX(INT_MIN, v, 0x4E, 0xF));
    v = imax_(v, DPPX(INT_MIN, v, 0x141, 0xF));
    v = imax_(v, DPPX(INT_MIN, v, 0x140, 0xF));
    v = imax_(v, DPPX(INT_MIN, v, 0x142, 0xA));
    v = imax_(v, DPPX(INT_MIN, v, 0x143, 0xC));
    return rdl(v, 63);
}
DEV i32 wave_min(i32 v) {
    v = imin_(v, DPPX(INT_MAX, v, 0xB1, 0xF));
    v = imin_(v, DPPX(INT_MAX, v, 0x4E, 0xF));
    v = imin_(v, DPPX(INT_MAX, v, 0x141, 0xF));
    v = imin_(v, DPPX(INT_MAX, v, 0x140, 0xF));
    v = imin_(v, DPPX(INT_MAX, v, 0x142, 0xA));
    v = imin_(v, DPPX(INT_MAX, v, 0x143, 0xC));
    return rdl(v, 63);
}
DEV i32 wave_sum(i32 v) {
    v = wadd(v, DPPX(0, v, 0xB1, 0xF));
    v = wadd(v, DPPX(0, v, 0x4E, 0xF));
    v = wadd(v, DPPX(0, v, 0x141, 0xF));
    v = wadd(v, DPPX(0, v, 0x140, 0xF));
    v = wadd(v, DPPX(0, v, 0x142, 0xA));
    v = wadd(v, DPPX(0, v, 0x143, 0xC));
    return rdl(v, 63);
}
// canonical float sum: xor-butterfly order 1, 2, 4, 8, 16, 32 (the C oracle
// emulates it bit for bit).  Done with DPP: quad_perm xor1 / xor2, then
// row_half_mirror and row_mirror (equal to xor4 / xor8 once each quad / half
// row holds one value; float + commutes exactly), then row_bcast15 / 31 into
// lane 63.  No LDS round trip.
#define FDPP(v, ctrl, rmask) __int_as_float(DPPX(0, __float_as_int(v), ctrl, rmask))
DEV float wave_fsum(float v) {
    v = v + FDPP(v, 0xB1, 0xF);
    v = v + FDPP(v, 0x4E, 0xF);
    v = v + FDPP(v, 0x141, 0xF);
    v = v + FDPP(v, 0x140, 0xF);
    v = v + FDPP(v, 0x142, 0xA);
    v = v + FDPP(v, 0x143, 0xC);
    return __int_as_float(rdl(__float_as_int(v), 63));
}
DEV unsigned long long ballot(bool p) { return __ballot(p); }
// A fresh copy of a uniform value: a comparison of it is then local to its one branch or
// select (s_cmp + s_cbranch_scc / s_cselect) instead of a comparison shared by several uses,
// which the compiler keeps as a 64-bit lane mask and tests with s_and_b64 exec at each use.
DEV i32 fresh(i32 v) {
    asm volatile("" : "+s"(v));
    return v;
}
// c ? a : b on two fields of a local struct, kept a select of VALUES: the compiler turns
// "select of two loads" into a load through a selected address, which puts the whole struct
// in scratch memory (64 lanes x its size of extra memory traffic per use)
DEV i32 sel(bool c, i32 a, i32 b) {
    asm volatile("" : "+v"(a));
    asm volatile("" : "+v"(b));
    return c ? a : b;
}
// pin a per-lane value in its VGPR: a chain of selects on it stays a chain of VALU selects
// (v_cmp + v_cndmask) instead of being folded into 64-bit lane-mask logic on the scalar unit
DEV u32 vkeep(u32 v) {
    asm volatile("" : "+v"(v));
    return v;
}
DEV float self(bool c, float a, float b) {  // (uniform floats live in VGPRs: the VALU computes them)
    asm volatile("" : "+v"(a));
    asm volatile("" : "+v"(b));
    return c ? a : b;
}

// Diagnostic build only (-DHFTLOB_STAMPS): per-phase shader-clock stamps of
// k_env_step, written to the info buffer in place of the info fields.
// STAMP marks the step's top phases, SUBSTAMP / STAMP_ACC the sub-phases; each read of the clock
// waits for the wave's outstanding scalar and LDS operations, so the sub-phase probes slow the
// phases they sit in: -DHFTLOB_STAMPS_COARSE keeps the top phases only (words 5..14 then 0).
#ifdef HFTLOB_STAMPS
#define STAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#ifdef HFTLOB_STAMPS_COARSE
#define SUBSTAMP(var) const unsigned long long var = 0
#define STAMP_ACC(acc, since)
#else
#define SUBSTAMP(var) STAMP(var)
#define STAMP_ACC(acc, since) acc += __builtin_amdgcn_s_memtime() - since
#endif
#else
#define STAMP(var)
#define SUBSTAMP(var)
#define STAMP_ACC(acc, since)
#endif

// ------------------------------------------------------------------ PRNG
DEV u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }
DEV void threefry(u32 k0, u32 k1, u32 x0, u32 x1, u32& o0, u32& o1) {
    const u32 k2 = k0 ^ k1 ^ 0x1BD11BDAu;
    x0 += k0;
    x1 += k1;
#define TF_R(r) x0 += x1; x1 = rotl32(x1, r); x1 ^= x0;
#define TF_G1 TF_R(13) TF_R(15) TF_R(26) TF_R(6)
#define TF_G2 TF_R(17) TF_R(29) TF_R(16) TF_R(24)
    TF_G1 x0 += k1; x1 += k2 + 1u;
    TF_G2 x0 += k2; x1 += k0 + 2u;
    TF_G1 x0 += k0; x1 += k1 + 3u;
    TF_G2 x0 += k1; x1 += k2 + 4u;
    TF_G1 x0 += k2; x1 += k0 + 5u;
#undef TF_G1
#undef TF_G2
#undef TF_R
    o0 = x0;
    o1 = x1;
}
struct Key { u32 a, b; };
// jax.random.split(key, n)[j]
DEV Key split_key(Key k, int n, int j, bool part) {
    Key o;
    if (part) { threefry(k.a, k.b, 0u, (u32)j, o.a, o.b); return o; }
    u32 y0, y1;
    int m = 2 * j;
    if (m < n) { threefry(k.a, k.b, (u32)m, (u32)(n + m), y0, y1); o.a = y0; }
    else { threefry(k.a, k.b, (u32)(m - n), (u32)m, y0, y1); o.a = y1; }
    m = 2 * j + 1;
    if (m < n) { threefry(k.a, k.b, (u32)m, (u32)(n + m), y0, y1); o.b = y0; }
    else { threefry(k.a, k.b, (u32)(m - n), (u32)m, y0, y1); o.b = y1; }
    return o;
}
// jax random_bits(key, 32, (n,))[i]
DEV u32 random_bits(Key k, int n, int i, bool part) {
    u32 y0, y1;
    if (part) { threefry(k.a, k.b, 0u, (u32)i, y0, y1); return y0 ^ y1; }
    int half = (n + 1) / 2;
    if (i < half) {
        threefry(k.a, k.b, (u32)i, (i + half < n) ? (u32)(i + half) : 0u, y0, y1);
        return y0;
    }
    threefry(k.a, k.b, (u32)(i - half), (i < n) ? (u32)i : 0u, y0, y1);
    return y1;
}
// jax.random.randint(key, (n,), lo, hi)[j], int32 (n = 1: the scalar draw)
DEV i32 randint_vec(Key k, int n, int j, i32 lo, i32 hi, bool part) {
    Key k1 = split_key(k, 2, 0, part), k2 = split_key(k, 2, 1, part);
    u32 hb = random_bits(k1, n, j, part), lb = random_bits(k2, n, j, part);
    u32 span = (hi <= lo) ? 1u : (u32)hi - (u32)lo;
    u32 mult = 65536u % span;
    mult = (mult * mult) % span;
    u32 off = ((hb % span) * mult + (lb % span)) % span;
    return (i32)((u32)lo + off);
}
// upper bound of the agent type's random action draw: Discrete(n_actions).sample, or
// MultiDiscrete([fixed_quant_value] * n_actions).sample for EXE fixed_prices (exec_env.py:2167-2171)
DEV i32 action_hi(const hftlob_agent_type_cfg& tc) {
    return tc.kind == HFTLOB_AGENT_EXE && tc.action_space == HFTLOB_EXE_ACT_FIXED_PRICES ? tc.fixed_quant_value
                                                                                         : tc.n_actions;
}
// jax.random.randint(key, (), lo, hi), int32
DEV i32 randint(Key k, i32 lo, i32 hi, bool part) { return randint_vec(k, 1, 0, lo, hi, part); }

// ------------------------------------------------------------ book tables
// Every table of the book (ask side, bid side, trade log) lives in LDS as
// structure-of-arrays: field f of slot s at base[f * R + s], R = the table's
// slot count.  A lane reads slots lane and lane+64 of one field with a
// conflict-free column load; one slot is read with a broadcast load and
// written by lanes 0..5 (one field each).  Keeping the book out of VGPRs
// removes the whole-book register copies the compiler emits at the control
// flow merges of the message dispatch, and LDS (8.4 KB per env for 100/100
// slots) keeps all 16 envs of a CU resident.
//
// Style rule for the hot path: lane predicates are built as 64-bit lane masks
// (v_cmp -> SGPR pair, combined with s_and/s_or), never as per-lane bool
// arrays or short-circuit && (which hipcc lowers to exec-masked branches).
struct LobCfg {
    i32 maxint, init_id, depth, cancel_mode, t4, check_fill, nO, nT;
};
DEV LobCfg lobcfg(const hftlob_lob_cfg& c) {
    LobCfg o;
    o.maxint = c.maxint; o.init_id = c.init_id; o.depth = c.book_depth; o.cancel_mode = c.cancel_mode;
    o.t4 = c.type_4_interpretation; o.check_fill = c.check_book_fill; o.nO = c.n_orders; o.nT = c.n_trades;
    return o;
}

typedef unsigned long long lmask;
DEV lmask bal(bool p) { return __builtin_amdgcn_ballot_w64(p); }
DEV int ffs64(lmask m) { return m ? (int)__builtin_ctzll(m) : -1; }

// v_writelane_b32 through the LLVM intrinsic (compiler-managed hazards)
extern "C" __device__ i32 __hftlob_writelane(i32 val, i32 lane, i32 old) __asm("llvm.amdgcn.writelane.i32");
DEV i32 wlane(i32 old, i32 val, int l) { return __hftlob_writelane(val, l, old); }

// Lanes of one wave exchange data through LDS without an s_barrier: every env workgroup is exactly
// one wave (the launch code's blocks of ENV_BLOCK = 64 threads, checked by one_wave() at each env
// kernel's entry), and a wave's LDS operations complete in issue order.  lds_order() keeps the
// compiler from moving an LDS access across a slot write of the message handlers (hot path);
// wave_sync() adds the wave-level scheduling barrier at the exchanges between phases (agent rows,
// _filter_messages, the shuffle, the no-op filter, the key batch).
#define ENV_BLOCK 64
DEV void lds_order() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }
DEV void wave_sync() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
}
DEV void one_wave() {  // the one-wave-per-workgroup assumption above
    if (blockDim.x != ENV_BLOCK) __builtin_trap();
}

enum { FP = 0, FQ, FOID, FTID, FTS, FTNS };  // order-side fields (JaxOrderBookArrays.py:21-28)

template <int S>
struct Valid {  // slot (or trade row) r*64+lane exists
    lmask m[S];
    bool v[S];
    DEV void init(int n) {
        const int l = lane_id();
#pragma unroll
        for (int r = 0; r < S; ++r) {
            // (the compiler does not know lane_id() < 64: state full register sets explicitly, so a
            // compile-time n folds them away)
            v[r] = (r + 1) * 64 <= n ? true : r * 64 + l < n;
            const int k = n - r * 64;
            m[r] = k >= 64 ? ~0ull : (k <= 0 ? 0ull : ((1ull << k) - 1ull));
        }
    }
};

// column load: o[r] = field f of slot r*64+lane (slots >= R read padding; mask with Valid)
template <int S> DEV void ldcol(const i32* t, int R, int f, i32 (&o)[S]) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) o[r] = t[f * R + r * 64 + l];
}
DEV i32 ldu(const i32* t, int R, int f, int e) { return uni(t[f * R + e]); }
// Slot writes: every lane stores, the lanes that are not writing a field
// store into their own word of a 64-word scratch row (`scr`).  That keeps
// the exec mask untouched (no s_and_saveexec / s_or pair per store), which
// matters because the scalar unit is the shared resource of a CU.
DEV void stu(i32* t, i32* scr, int R, int f, int e, i32 v) {
    const int l = lane_id();
    *(l == 0 ? t + f * R + e : scr + l) = v;
    lds_order();
}
DEV void st6(i32* t, i32* scr, int R, int e, i32 f0, i32 f1, i32 f2, i32 f3, i32 f4, i32 f5) {
    const int l = lane_id();
    i32 v = f0;
    v = wlane(v, f1, 1); v = wlane(v, f2, 2); v = wlane(v, f3, 3); v = wlane(v, f4, 4); v = wlane(v, f5, 5);
    *(l < 6 ? t + l * R + e : scr + l) = v;
    lds_order();
}
DEV void clr6(i32* t, i32* scr, int R, int e) {
    const int l = lane_id();
    *(l < 6 ? t + l * R + e : scr + l) = -1;
    lds_order();
}
// s_ff1_i32_b64: index of the lowest set bit, -1 (all ones) for an empty mask
DEV u32 ff1(lmask m) {
    u32 r;
    asm("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m));
    return r;
}
// first slot over per-register lane masks; `fallback` if none.  An empty
// register's -1 survives `| 64*r` and loses every unsigned min.
template <int S> DEV int first_slot(const lmask (&m)[S], int fallback) {
    u32 idx = ff1(m[0]);
#pragma unroll
    for (int r = 1; r < S; ++r) idx = min(idx, ff1(m[r]) | (u32)(64 * r));
    return idx == 0xFFFFFFFFu ? fallback : (int)idx;
}
template <int S> DEV int first_true(const bool (&pr)[S], int fallback) {
    lmask m[S];
#pragma unroll
    for (int r = 0; r < S; ++r) m[r] = bal(pr[r]);
    return first_slot(m, fallback);
}
// value of (uniform) slot e from a column held lane-strided in registers
template <int S> DEV i32 sget(const i32 (&a)[S], int e) {
    i32 v = a[0];  // pick the register set (v_cndmask on a uniform condition), then one v_readlane
#pragma unroll
    for (int k = 1; k < S; ++k) v = (e >> 6) == k ? a[k] : v;
    return rdl(v, e & 63);
}

template <int S>
struct Side {
    i32* t;              // LDS table [6][R]
    i32* scr;            // LDS scratch row (64 words)
    i32 best_p, best_q;  // get_best_{ask,bid} price and get_volume_at_price(best); valid unless F_STALE
    i32 xp;              // asks: the best price a bid crosses against (an empty side: maxint), with best_p
    i32 pc[S];           // the price column, lane-strided in VGPRs (a write-through copy of field FP):
                         // every handler reads prices, only adds and row clears write them
    // top-of-book cache: the slot _get_top_*_order_idx returns for max / min price top_p, and its
    // (ts, tns); top = -1: unknown.  Kept across messages: a quantity change keeps it, clearing the
    // row (or any bulk clear) drops it, an add at a better price or an earlier time at top_p
    // replaces it (see top_new / top_eq), so a crossing message usually skips the top-of-book scan
    i32 top, top_p, top_ts, top_tns;
    // the chunk's best-quote record of this side (run_chunk): lane k holds (best_p, best_q) after
    // message k if the message set or recomputed them (lane k of rm), else the lanes are filled
    // from the last recording lane before them when the chunk ends
    i32 rp, rq;
    lmask rm;
};
// a message (its lane k of the chunk) set or recomputed the side's best quote: record it
template <int S> DEV void side_rec(Side<S>& s, u32 k) {
    s.rp = wlane(s.rp, s.best_p, (int)k);
    s.rq = wlane(s.rq, s.best_q, (int)k);
    asm volatile("s_bitset1_b64 %0, %1" : "+s"(s.rm) : "s"(k));
}

// slot e of a lane-strided register column <- v (lane e & 63 of register e >> 6): one
// compare and one select per register set, no scalar work
template <int S> DEV void col_set(i32 (&c)[S], int e, i32 v) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) c[r] = (l + 64 * r == e) ? v : c[r];
}

// Wave-uniform book flags, one SGPR bitfield (bools would each be a 64-bit
// lane mask the compiler copies at every merge):
//   STALE  the side's cached best quote must be recomputed; STALE_ANY is set with either
//          side's bit (SideBits::MARK), so the test after each message is one bit test
//   CLEAN  every row with q <= 0 is an all -1 row => _removeZeroNegQuant only
//          ever has to look at the row just written
//   NEG1   some row with p != -1 holds a -1 in another field (then "first row
//          holding ANY -1" needs the full test, else p == -1 suffices)
//   PM1    some row with p == -1 holds a field != -1 (an order priced -1)
//   SLOW   not FAST.  FAST: both sides CLEAN, neither NEG1 nor PM1 (the handlers' common
//          variant): then a row holds a -1 <=> its price is -1 <=> it is all -1, so the free
//          slots are the p == -1 slots of the register price column.  The sign bit: the
//          per-message variant test (i32)fl < 0 is one s_cmp_lt_i32
// (bit 0 is left unused: a branch on a bit-0 test compiles to s_bitcmp1 + a 64-bit lane mask
// + s_and_b64 exec + s_cbranch_vccnz, on any other bit to s_bitcmp1 + s_cbranch_scc)
enum : u32 { F_STALE_A = 2, F_STALE_B = 4, F_CLEAN_A = 8, F_CLEAN_B = 16, F_NEG1_A = 32, F_NEG1_B = 64,
             F_PM1_A = 256, F_PM1_B = 512, F_STALE_ANY = 0x40000000u, F_SLOW = 0x80000000u };
constexpr u32 STALE_ANY = F_STALE_ANY;  // set with either side's STALE bit: one bit test after each message
template <bool ASKS> struct SideBits {
    static constexpr u32 STALE = ASKS ? F_STALE_A : F_STALE_B;
    static constexpr u32 MARK = STALE | STALE_ANY;  // (sets STALE)
    static constexpr u32 CLEAN = ASKS ? F_CLEAN_A : F_CLEAN_B;
    static constexpr u32 NEG1 = ASKS ? F_NEG1_A : F_NEG1_B;
    static constexpr u32 PM1 = ASKS ? F_PM1_A : F_PM1_B;
};
DEV u32 slow_bit(u32 fl) {
    return (fl & (F_CLEAN_A | F_CLEAN_B | F_NEG1_A | F_NEG1_B | F_PM1_A | F_PM1_B)) == (F_CLEAN_A | F_CLEAN_B)
               ? 0u : F_SLOW;
}

// A side's rows in registers between the global load and the LDS commit, so
// the HBM latency of the load can overlap other work.
template <int S>
struct SideRows {
    int2 x0[S], x1[S], x2[S];  // (p, q), (oid, tid), (ts, tns) of slot r*64+lane
};
template <int S> DEV void fetch_side(SideRows<S>& f, const i32* g, const Valid<S>& V) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        f.x0[r] = f.x1[r] = f.x2[r] = make_int2(-1, -1);
        if (V.v[r]) {
            const int2* row = reinterpret_cast<const int2*>(g + (r * 64 + l) * 6);
            f.x0[r] = row[0]; f.x1[r] = row[1]; f.x2[r] = row[2];
        }
    }
}
// fetched rows -> LDS side table; returns the side's CLEAN / NEG1 bits.  The per-row "any field
// == -1" / "all fields == -1" tests run as unsigned min / max of the complemented fields (VALU),
// not as chains of lane-mask logic.
template <bool ASKS, int S>
DEV u32 commit_side(Side<S>& s, const SideRows<S>& f, int R, const Valid<S>& V) {
    const int l = lane_id();
    lmask bad = 0, n1 = 0, pm1 = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const int sl = r * 64 + l;
        const i32 p = f.x0[r].x, q = f.x0[r].y, oid = f.x1[r].x, tid = f.x1[r].y, ts = f.x2[r].x, tns = f.x2[r].y;
        if (V.v[r]) {
            i32* t = s.t + sl;
            t[FP * R] = p; t[FQ * R] = q; t[FOID * R] = oid; t[FTID * R] = tid; t[FTS * R] = ts; t[FTNS * R] = tns;
        }
        s.pc[r] = V.v[r] ? p : -1;
        const u32 np_ = ~(u32)p, nq = ~(u32)q, no = ~(u32)oid, nt = ~(u32)tid, ns = ~(u32)ts, nn = ~(u32)tns;
        const u32 any0 = min(min(min(np_, nq), min(no, nt)), min(ns, nn));  // 0 <=> some field == -1
        const u32 all0 = max(max(max(np_, nq), max(no, nt)), max(ns, nn));  // 0 <=> every field == -1
        bad |= V.m[r] & bal((q <= 0) & (all0 != 0u));
        n1 |= V.m[r] & bal((p != -1) & (any0 == 0u));
        pm1 |= V.m[r] & bal((p == -1) & (all0 != 0u));
    }
    lds_order();
    s.top = -1;
    return (bad == 0ull ? SideBits<ASKS>::CLEAN : 0u) | (n1 != 0ull ? SideBits<ASKS>::NEG1 : 0u) |
           (pm1 != 0ull ? SideBits<ASKS>::PM1 : 0u);
}
// a side whose table is already in LDS (k_env_rollout: the wave's previous step left it there,
// and its flags): the register price column from the table
template <int S> DEV void relink_side(Side<S>& s, int R, const Valid<S>& V) {
    i32 p[S];
    ldcol(s.t, R, FP, p);
#pragma unroll
    for (int r = 0; r < S; ++r) s.pc[r] = V.v[r] ? p[r] : -1;
    s.top = -1;
}
template <bool ASKS, int S> DEV u32 load_side(Side<S>& s, const i32* g, int R, const Valid<S>& V) {
    SideRows<S> f;
    fetch_side(f, g, V);
    return commit_side<ASKS>(s, f, R, V);
}
template <int S> DEV void store_side(const Side<S>& s, i32* g, int R, const Valid<S>& V) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const int sl = r * 64 + l;
        if (V.v[r]) {
            const i32* t = s.t + sl;
            int2* row = reinterpret_cast<int2*>(g + sl * 6);
            row[0] = make_int2(t[FP * R], t[FQ * R]);
            row[1] = make_int2(t[FOID * R], t[FTID * R]);
            row[2] = make_int2(t[FTS * R], t[FTNS * R]);
        }
    }
}
// clear every valid slot selected by lane mask m (the LDS rows and the register price column)
template <int S> DEV void clear_masked(Side<S>& s, int R, const lmask (&m)[S]) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const bool hit = (m[r] >> l) & 1ull;
        s.pc[r] = hit ? -1 : s.pc[r];
        if (hit) {
#pragma unroll
            for (int f = 0; f < 6; ++f) s.t[f * R + r * 64 + l] = -1;
        }
    }
    lds_order();
    s.top = -1;
}

// _removeZeroNegQuant — JaxOrderBookArrays.py:85-90 on a side that is not
// clean (on a clean side only the row just written can hold q <= 0, and the
// handlers clear it directly)
template <bool ASKS, int S> DEV void rzn(Side<S>& s, u32& fl, int R, const Valid<S>& V) {
    i32 q[S];
    ldcol(s.t, R, FQ, q);
    lmask m[S];
#pragma unroll
    for (int r = 0; r < S; ++r) m[r] = V.m[r] & bal(q[r] <= 0);
    clear_masked(s, R, m);
    fl = fl | SideBits<ASKS>::CLEAN | SideBits<ASKS>::MARK;
    fl = (fl & ~F_SLOW) | slow_bit(fl);
}

// get_best_bid: max raw price (empty side -> -1); volume at it — :943-951,906-917
template <int S> DEV void best_bid_pq(const i32 (&p)[S], const i32 (&q)[S], const Valid<S>& V, i32& bp, i32& bq) {
    i32 m = INT_MIN;
#pragma unroll
    for (int r = 0; r < S; ++r) m = imax_(m, V.v[r] ? p[r] : INT_MIN);
    const i32 mp = wave_max(m);
    i32 v = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) v = wadd(v, (V.v[r] & (p[r] == mp)) ? q[r] : 0);
    bp = mp;
    bq = wave_sum(v);
}
// get_best_ask: min price with -1 -> maxint, maxint -> -1; volume at it — :932-941
template <int S>
DEV void best_ask_pq(const i32 (&p)[S], const i32 (&q)[S], const Valid<S>& V, i32 maxint, i32& bp, i32& bq,
                     i32* xp = nullptr) {
    i32 m = INT_MAX;
#pragma unroll
    for (int r = 0; r < S; ++r) m = imin_(m, V.v[r] ? (p[r] == -1 ? maxint : p[r]) : INT_MAX);
    const i32 mn = wave_min(m);
    if (xp) *xp = mn;  // (== pa, or maxint for an empty side or a maxint-only one: pa -1)
    const i32 pa = mn == maxint ? -1 : mn;
    i32 v = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) v = wadd(v, (V.v[r] & (p[r] == pa)) ? q[r] : 0);
    bp = pa;
    bq = wave_sum(v);
}
// recompute a side's cached best quote (clears its STALE bit); REC: inside message k's
// processing, which then records the quote
template <bool ASKS, bool REC, int S>
DEV void rescan(Side<S>& s, u32& fl, int R, const Valid<S>& V, i32 maxint, u32 k) {
    i32 q[S];
    ldcol(s.t, R, FQ, q);
    if (ASKS) best_ask_pq(s.pc, q, V, maxint, s.best_p, s.best_q, &s.xp);
    else best_bid_pq(s.pc, q, V, s.best_p, s.best_q);
    fl &= ~SideBits<ASKS>::STALE;
    if (REC) side_rec(s, k);
}

// _get_top_bid_order_idx / _get_top_ask_order_idx — :241-268 (exact formulas);
// mp is the side's max price (bid) / min price with -1 -> maxint (ask)
template <int S>
DEV int top_idx(const i32 (&p)[S], const i32 (&ts)[S], const i32 (&tns)[S], const Valid<S>& V, const LobCfg& c, i32 mp,
                i32& mts_out, i32& mtn_out) {
    i32 t[S], n[S], m = INT_MAX;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        t[r] = (p[r] == mp) ? ts[r] : c.maxint;
        m = imin_(m, V.v[r] ? t[r] : INT_MAX);
    }
    const i32 mts = wave_min(m);
    m = INT_MAX;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        n[r] = (t[r] == mts) ? tns[r] : c.maxint;
        m = imin_(m, V.v[r] ? n[r] : INT_MAX);
    }
    const i32 mtn = wave_min(m);
    mts_out = mts;
    mtn_out = mtn;
    lmask pm[S];
#pragma unroll
    for (int r = 0; r < S; ++r) pm[r] = V.m[r] & bal(n[r] == mtn);
    return first_slot(pm, c.nO - 1);
}

// ------------------------------------------------------------ trade log
// LDS table [8 fields][R = nT rows]; appends (rare) touch one row.
struct Trades {
    i32* t;
    i32* scr;
    int R;
    DEV i32 get(int k, int r) const { return t[k * R + r * 64 + lane_id()]; }
    DEV i32 at(int k, int row) const { return uni(t[k * R + row]); }
};
template <int S> DEV void trades_fill(Trades& T, const Valid<S>& V, i32 v) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r)
        if (V.v[r]) {
#pragma unroll
            for (int k = 0; k < 8; ++k) T.t[k * T.R + r * 64 + l] = v;
        }
    lds_order();
}
template <int S> DEV void load_trades(Trades& T, const i32* g, const Valid<S>& V) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        if (V.v[r]) {
            const int o = r * 64 + l, R = T.R;
            const int4* row = reinterpret_cast<const int4*>(g + o * 8);
            const int4 a = row[0], b = row[1];
            T.t[0 * R + o] = a.x; T.t[1 * R + o] = a.y; T.t[2 * R + o] = a.z; T.t[3 * R + o] = a.w;
            T.t[4 * R + o] = b.x; T.t[5 * R + o] = b.y; T.t[6 * R + o] = b.z; T.t[7 * R + o] = b.w;
        }
    }
    lds_order();
}
template <int S> DEV void store_trades(const Trades& T, i32* g, const Valid<S>& V) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        if (V.v[r]) {
            const int o = r * 64 + l, R = T.R;
            int4* row = reinterpret_cast<int4*>(g + o * 8);
            row[0] = make_int4(T.t[0 * R + o], T.t[1 * R + o], T.t[2 * R + o], T.t[3 * R + o]);
            row[1] = make_int4(T.t[4 * R + o], T.t[5 * R + o], T.t[6 * R + o], T.t[7 * R + o]);
        }
    }
}
// write trade row e (uniform) — lanes 0..7 store one field each
DEV void trade_put(Trades& T, int e, i32 f0, i32 f1, i32 f2, i32 f3, i32 f4, i32 f5, i32 f6, i32 f7) {
    const int l = lane_id();
    i32 v = f0;
    v = wlane(v, f1, 1); v = wlane(v, f2, 2); v = wlane(v, f3, 3);
    v = wlane(v, f4, 4); v = wlane(v, f5, 5); v = wlane(v, f6, 6); v = wlane(v, f7, 7);
    *(l < 8 ? T.t + l * T.R + e : T.scr + l) = v;
    lds_order();
}

// ------------------------------------------------------ message handlers
// G (general) = false instantiates the handlers for the common case where
// both sides are clean and neg1-free (flags that only add_order can change):
// the kernels run that variant while F_SLOW is clear.
template <int S>
struct Book {
    Side<S> a, b;
    Trades tr;
    Valid<S> vs, vt;
    LobCfg c;
    u32 fl;  // F_* bits
    // cancel_mode 2/3 only (RC instantiations): the scan's key and the index
    // of the message being processed (keys = split(ek, nmsg); key i is message i's)
    Key ek;
    i32 mi, nmsg;
    // trade log: rows [0, ntr) hold col 4 != -1, rows [ntr, nT) col 4 == -1, so the next trade
    // goes to row min(ntr, nT - 1) (match_order's "first row whose col 4 == -1", -1 -> last row).
    // -1: the log loaded from memory has no such prefix shape; match_order then searches it.
    i32 ntr;
    bool part;
    i32* filt;  // LDS: the 2048-bit id / init-price filter of chunk_noops (64 words)
    // the filter already holds a superset of the book's ids and init-id rows (built at an earlier
    // chunk of this step, plus every add id since): the next chunk only inserts its own add ids
    bool filt_ok;
};

// message handler codes (the reference's dispatch index) and flags, see decode_msgs
enum { H_ASK = 0, H_BID = 1, H_CNL_ASK = 2, H_CNL_BID = 3, H_NOP = 4, H_KIND = 7, H_DISCARD = 8, H_NEG1 = 16,
       H_PM1 = 32, H_MKT = 64, H_RARE = 128 };
struct Msg {
    i32 h, side, price, qty, oid, tid, t, tns;  // h: handler code and H_* flags (decode_msgs)
    u32 k;                                      // its lane in the chunk (the best-quote record's)
};

// Incremental best-quote bookkeeping.  Every update below is exact for a clean
// side: it changes (best_p, best_q) only where get_best_* / get_volume_at_price
// would, and falls back to a full recompute (ok = false) where it cannot tell.
// the top-of-book cache after an order (np, t, tns) went to slot e:
// a new best price: the row is alone at it, so it is the top (unless a maxint time, where the
// top-of-book formula's maxint placeholders could tie with it)
template <int S> DEV void top_new(Side<S>& s, int e, i32 np, i32 t, i32 tns, i32 maxint) {
    s.top = ((t != maxint) & (tns != maxint)) ? e : -1;
    s.top_p = np; s.top_ts = t; s.top_tns = tns;
}
// an order at the best price: the top moves to it only if it is earlier in (ts, tns, slot)
// (a known top is at the best price, np: note_add drops it whenever the best quote is not known;
// one branch per test, the common case first: an OR of the tests becomes 64-bit lane-mask logic
// on the scalar unit)
template <int S> DEV void top_eq(Side<S>& s, int e, i32 t, i32 tns, i32 maxint) {
    if (fresh(t) > s.top_ts) return;  // a later order (the common case)
    asm volatile("");
    if (s.top < 0) return;
    asm volatile("");
    bool earlier = t < s.top_ts;
    if (!earlier) earlier = (tns < s.top_tns) | ((tns == s.top_tns) & (e < s.top));
    if (earlier) {
        s.top = tns != maxint ? e : -1;  // (t < top_ts < maxint)
        s.top_ts = t; s.top_tns = tns;
    }
}
// STALE_OK = false: the caller knows the side is not stale (add_free: no message starts with a
// stale side, run_chunk refreshes both after each one, and an add without eviction changes only
// the other side before it gets here)
#define XP_SET(s, v) ((s).xp = (v))  // (asks: a new best price below maxint)
// NN: np >= 0 is known (the common adds: decode_msgs marks negative prices RARE)
template <bool BID, int S, bool STALE_OK = true, bool NN = false>
DEV void note_add(Side<S>& s, u32& fl, int e, i32 np, i32 nq, i32 t, i32 tns, i32 maxint, u32 k) {
    // an all -1 row (slot e) now holds (np, nq > 0, time t / tns).  Branches ordered for the
    // common case, an order behind the best (one compare each); per side the cases are those of
    // get_best_* with -1 (and, for asks, maxint) standing for "no price".
    constexpr u32 STALE = SideBits<!BID>::STALE, MARK = SideBits<!BID>::MARK;
    if (STALE_OK && (fl & STALE)) { s.top = -1; return; }
    const i32 bp = s.best_p;
    if (BID) {
        if (np < bp) {
            if (!NN && bp == -1) fl |= MARK;  // np < -1 on an empty side
        } else if (np > bp) {
            s.best_p = np; s.best_q = nq;   // (an empty side: np > -1)
            side_rec(s, k);
            top_new(s, e, np, t, tns, maxint);
        } else if (!NN && bp == -1) {
            fl |= MARK;                       // np == -1 on an empty side
        } else {
            s.best_q = wadd(s.best_q, nq);
            side_rec(s, k);
            top_eq(s, e, t, tns, maxint);
        }
    } else {
        if (np > bp) {
            if (bp == -1) {                 // empty side
                if (np == maxint) fl |= MARK;
                else { s.best_p = np; s.best_q = nq; XP_SET(s, np); side_rec(s, k); top_new(s, e, np, t, tns, maxint); }
            }
        } else if (np < bp) {
            if (NN || np != -1) { s.best_p = np; s.best_q = nq; XP_SET(s, np); side_rec(s, k); top_new(s, e, np, t, tns, maxint); }
        } else if (!NN && np == -1) {
            fl |= MARK;
        } else if (np != maxint) {
            s.best_q = wadd(s.best_q, nq);
            side_rec(s, k);
            top_eq(s, e, t, tns, maxint);
        }
    }
}
// a row at price op lost dq of its quantity (possibly all of it)
template <bool ASKS, int S> DEV void note_reduce(Side<S>& s, u32& fl, i32 op, i32 dq, u32 k) {
    constexpr u32 STALE = SideBits<ASKS>::STALE, MARK = SideBits<ASKS>::MARK;
    if (fl & STALE) return;
    if (op == s.best_p) {
        if (op == -1) {
            fl |= MARK;
        } else {
            s.best_q = wsub(s.best_q, dq);
            side_rec(s, k);
            if (s.best_q <= 0) fl |= MARK;  // level exhausted (or odd data): rescan
        }
    } else {
        // a row behind the best: the quote stands unless a -1 price is involved (scalar selects;
        // as one branch on "op == -1 || best == -1" the compiler builds 64-bit lane masks)
        asm volatile("");
        u32 f = fl;
        f = fresh(op) == -1 ? f | MARK : f;
        f = fresh(s.best_p) == -1 ? f | MARK : f;
        fl = f;
    }
}

// row writes that keep the register price column in step with field FP
template <int S> DEV void side_put(Side<S>& s, int R, int e, i32 f0, i32 f1, i32 f2, i32 f3, i32 f4, i32 f5) {
    st6(s.t, s.scr, R, e, f0, f1, f2, f3, f4, f5);
    col_set(s.pc, e, f0);
}
template <int S> DEV void side_clr(Side<S>& s, int R, int e) {
    clr6(s.t, s.scr, R, e);
    col_set(s.pc, e, -1);
    s.top = e == s.top ? -1 : s.top;
}
// the side's p == -1 slots (all -1 rows in the FAST variant)
template <int S> DEV void free_slots(const Book<S>& B, const Side<S>& s, lmask (&free)[S]) {
#pragma unroll
    for (int r = 0; r < S; ++r) free[r] = B.vs.m[r] & bal(s.pc[r] == -1);
}

template <int S> DEV bool no_slot(const lmask (&m)[S]) {
    lmask a = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) a |= m[r];
    return a == 0ull;
}

// match_order — JaxOrderBookArrays.py:172-220
// (qt, pt, ot, tt): the top slot's quantity, price, order id, trader id;
// tr4: the trade log's OID column
template <bool G, bool ASKS, int S>
DEV i32 match_order(Book<S>& B, Side<S>& s, int top, i32 qtm, const Msg& m, i32 qt, i32 pt, i32 ot, i32 tt) {
    const int R = B.c.nO;
    const i32 newq = imax_(0, wsub(qt, qtm));
    const i32 rem = wsub(qtm, qt);
    int e;
    if (B.ntr >= 0) {  // the row after the last written one; a trade whose col 4 (the message time,
                       // TradesFeat SEC) is -1 leaves its row free for the next trade
        e = imin_(B.ntr, B.c.nT - 1);
        if (m.t != -1) B.ntr = imin_(B.ntr + 1, B.c.nT);
    } else {
        i32 tr4[S];
        ldcol(B.tr.t, B.tr.R, 4, tr4);
        lmask fm[S];
#pragma unroll
        for (int r = 0; r < S; ++r) fm[r] = B.vt.m[r] & bal(tr4[r] == -1);  // trade[:,OID=4] == -1
        e = first_slot(fm, B.c.nT - 1);
    }
    trade_put(B.tr, e, pt, wmul(wsub(0, m.side), wsub(qt, newq)), ot, m.oid, m.t, m.tns, tt, m.tid);
    if (!G || (B.fl & SideBits<ASKS>::CLEAN)) {
        if (newq <= 0) side_clr(s, R, top);
        else stu(s.t, s.scr, R, FQ, top, newq);
        note_reduce<ASKS>(s, B.fl, pt, wsub(qt, newq), m.k);
    } else {
        stu(s.t, s.scr, R, FQ, top, newq);
        rzn<ASKS>(s, B.fl, R, B.vs);
    }
    return rem;
}

// _match_against_{bid,ask}_orders — :284-331.  The top slot's price never
// beats the side's best, so "best does not cross" ends the loop exactly; only
// a crossing best pays for the 3-reduction top-of-book.
// a crossing trip loads every column it needs at once (one LDS round trip)
// POS: qtm > 0 is known (the common FAST adds, decode_msgs)
template <bool BID, bool G, int S, bool POS = false>
DEV i32 match_against(Book<S>& B, Side<S>& s, i32 qtm, i32 price, const Msg& m) {
    const int R = B.c.nO;
    // the common case first, as straight-line scalar code: nothing to match, or a best that
    // does not cross (the loop's own first test, with an empty ask side standing for maxint)
    // (fresh: the RARE / common handler copies each keep their own test, not one shared lane mask)
    if (!POS && fresh(qtm) <= 0) return qtm;
    // (no stale side here: run_chunk refreshes both sides after every message)
    {
        const i32 bp = s.best_p;
        const i32 mp0 = (!BID && bp == -1) ? B.c.maxint : bp;
        if (__builtin_expect(BID ? mp0 < price : mp0 > price, 1)) return qtm;
    }
    while (qtm > 0) {
        if (B.fl & SideBits<!BID>::STALE) rescan<!BID, true>(s, B.fl, R, B.vs, B.c.maxint, m.k);
        // the side's best; an empty ask side (-1) counts as maxint (_get_top_ask_order_idx).
        // BID: `s` is the bid side (an incoming sell crosses when best bid >= price)
        i32 mp = s.best_p;
        if (!BID) {
            if (mp == -1) {
                if (price != B.c.maxint) break;
                mp = B.c.maxint;
            } else if (mp > price) {
                break;
            }
        } else if (mp < price) {
            break;
        }
        int top;
        i32 qt, ot, tt, tp;
        if (s.top >= 0 && s.top_p == mp) {  // the cached top (a row at mp): three broadcast reads
            top = s.top;
            qt = ldu(s.t, R, FQ, top); ot = ldu(s.t, R, FOID, top); tt = ldu(s.t, R, FTID, top);
            tp = mp;
        } else {
            i32 q[S], o[S], t[S], ts[S], tn[S], mts, mtn;
            ldcol(s.t, R, FTS, ts); ldcol(s.t, R, FTNS, tn);
            ldcol(s.t, R, FQ, q); ldcol(s.t, R, FOID, o); ldcol(s.t, R, FTID, t);
            top = top_idx(s.pc, ts, tn, B.vs, B.c, mp, mts, mtn);
            qt = sget(q, top); ot = sget(o, top); tt = sget(t, top); tp = sget(s.pc, top);
            s.top_p = mp; s.top_ts = mts; s.top_tns = mtn;
            // cached only when the formula picks the earliest row AT mp: if the earliest-ts rows
            // at mp all have tns == maxint, the formula's maxint placeholders tie and it returns
            // the side's first slot, whatever its price or time (a quirk kept bit for bit, which
            // tests/streams.py::top_streams reaches)
            s.top = ((tp == mp) & (mp != -1) & (mp != B.c.maxint) & (mts != B.c.maxint) & (mtn != B.c.maxint))
                        ? top : -1;
        }
        if (fresh(tp) == -1) break;  // (two branches, not a 64-bit lane-mask OR)
        asm volatile("");
        if (BID ? tp < price : tp > price) break;
        qtm = match_order<G, !BID>(B, s, top, qtm, m, qt, tp, ot, tt);
    }
    return qtm;
}

// add_order — :62-83 (first slot holding ANY -1 field; none -> last slot)
// free: the side's p == -1 slots (from the caller)
template <bool BID, bool G, int S>
DEV void add_order(Book<S>& B, Side<S>& s, const Msg& m, i32 qty, const lmask (&free)[S]) {
    const int R = B.c.nO;
    constexpr u32 CLEAN = SideBits<!BID>::CLEAN, NEG1 = SideBits<!BID>::NEG1, MARK = SideBits<!BID>::MARK,
                  PM1 = SideBits<!BID>::PM1;
    const i32 nq = imax_(0, qty);
    if (!G) {  // FAST: "any -1" <=> p == -1 <=> an all -1 row; no free slot -> the last slot, which holds an order
        const int e = first_slot(free, R - 1);
        const bool was_empty = !no_slot(free);
        if (nq > 0) {
            side_put(s, R, e, m.price, nq, m.oid, m.tid, m.t, m.tns);
            if (m.h & (H_NEG1 | H_PM1)) B.fl = B.fl | (m.h & H_NEG1 ? NEG1 : 0u) | (m.h & H_PM1 ? PM1 : 0u) | F_SLOW;
            if (was_empty) note_add<BID>(s, B.fl, e, m.price, nq, m.t, m.tns, B.c.maxint, m.k);
            else { B.fl |= MARK; s.top = -1; }
        } else if (!was_empty) {  // the new row is removed at once: net effect clears row e
            side_clr(s, R, e);
            B.fl |= MARK;
        }
        return;
    }
    lmask fm[S];
    i32 q[S];
    ldcol(s.t, R, FQ, q);
    if ((B.fl & (CLEAN | NEG1 | PM1)) == CLEAN) {  // then "any -1" <=> p == -1
#pragma unroll
        for (int r = 0; r < S; ++r) fm[r] = free[r];
    } else {
        i32 o[S], t[S], ts[S], tn[S];
        ldcol(s.t, R, FOID, o); ldcol(s.t, R, FTID, t);
        ldcol(s.t, R, FTS, ts); ldcol(s.t, R, FTNS, tn);
#pragma unroll
        for (int r = 0; r < S; ++r)
            fm[r] = B.vs.m[r] & (bal(s.pc[r] == -1) | bal(q[r] == -1) | bal(o[r] == -1) | bal(t[r] == -1) |
                                 bal(ts[r] == -1) | bal(tn[r] == -1));
    }
    const int e = first_slot(fm, R - 1);
    if (!(B.fl & CLEAN)) {  // stray q<=0 rows: write, then the full _removeZeroNegQuant
        side_put(s, R, e, m.price, nq, m.oid, m.tid, m.t, m.tns);
        if (m.h & H_PM1) B.fl |= PM1;
        rzn<!BID>(s, B.fl, R, B.vs);
        return;
    }
    const i32 op = sget(s.pc, e), oq = sget(q, e);
    const bool was_empty = (op == -1) & (oq == -1);  // clean: q == -1 <=> all -1 row
    if (nq > 0) {
        side_put(s, R, e, m.price, nq, m.oid, m.tid, m.t, m.tns);
        if (m.h & H_NEG1) B.fl |= NEG1;
        if (m.h & H_PM1) B.fl |= PM1;
        if (was_empty) note_add<BID>(s, B.fl, e, m.price, nq, m.t, m.tns, B.c.maxint, m.k);
        else { B.fl |= MARK; s.top = -1; }
    } else if (!was_empty) {  // the new row is removed at once: net effect clears row e
        side_clr(s, R, e);
        B.fl |= MARK;
    }
}

// check_book_fill eviction — :395-401 (bid: worst = min), :484-490 (ask: max);
// called when no slot holds p == -1: evicts only if every price is >= 0
template <bool BID, int S> DEV void evict_if_full(Book<S>& B, Side<S>& s, lmask (&free)[S]) {
    const int R = B.c.nO;
    lmask neg = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) neg |= B.vs.m[r] & bal(s.pc[r] < 0);
    if (neg != 0ull) return;
    i32 w = BID ? INT_MAX : INT_MIN;
#pragma unroll
    for (int r = 0; r < S; ++r)
        w = BID ? imin_(w, B.vs.v[r] ? s.pc[r] : INT_MAX) : imax_(w, B.vs.v[r] ? s.pc[r] : INT_MIN);
    const i32 worst = BID ? wave_min(w) : wave_max(w);
    lmask m[S];
#pragma unroll
    for (int r = 0; r < S; ++r) m[r] = B.vs.m[r] & bal(s.pc[r] == worst);
    const i32 top = s.top;
    clear_masked(s, R, m);
    // only the worst level goes: the best quote and the top of book survive unless the side holds
    // one price level (worst == best; an ask side whose prices are all maxint has best -1)
    s.top = worst != s.top_p ? top : -1;
    if ((worst == s.best_p) | (s.best_p == -1)) B.fl |= SideBits<!BID>::MARK;
    free_slots(B, s, free);
}
// The common add: FAST book, a free (all -1) slot exists, no eviction: the order goes to the
// first free slot (add_order's "first row holding any -1").  Flag changes are rare (orders with
// -1 fields), so they stay behind a branch.
// POS: qty > 0 is known (the common add that does not cross)
template <bool BID, bool RARE, int S, bool POS = false>
DEV void add_free(Book<S>& B, Side<S>& s, const Msg& m, i32 qty, const lmask (&free)[S]) {
    const int R = B.c.nO;
    if (!POS && qty <= 0) return;  // imax(0, qty) == 0: the new row is removed at once and the slot was empty
    u32 e;
    if (S == 2) {  // the slot's register set is known from the branch: one v_writelane updates the price column
        if (free[0] != 0ull) {
            e = ff1(free[0]);
            s.pc[0] = wlane(s.pc[0], m.price, (int)e);
        } else {
            e = ff1(free[S - 1]);
            s.pc[S - 1] = wlane(s.pc[S - 1], m.price, (int)e);
            e |= 64u;
        }
        st6(s.t, s.scr, R, (int)e, m.price, qty, m.oid, m.tid, m.t, m.tns);
    } else {
        e = ff1(free[0]);
#pragma unroll
        for (int r = 1; r < S; ++r) e = min(e, ff1(free[r]) | (u32)(64 * r));
        side_put(s, R, (int)e, m.price, qty, m.oid, m.tid, m.t, m.tns);
    }
    if (RARE && __builtin_expect((m.h & (H_NEG1 | H_PM1)) != 0, 0)) {
        // rare: kept as a branch (the empty asm stops if-conversion into ~10 scalar selects per add)
        asm volatile("");
        constexpr u32 NEG1 = SideBits<!BID>::NEG1, PM1 = SideBits<!BID>::PM1;
        B.fl = B.fl | (m.h & H_NEG1 ? NEG1 : 0u) | (m.h & H_PM1 ? PM1 : 0u) | F_SLOW;
    }
    note_add<BID, S, false, !RARE>(s, B.fl, (int)e, m.price, qty, m.t, m.tns, B.c.maxint, m.k);
}
// bid_lim — :357-420 (the eviction persists when the add is discarded)
// RARE = false: the message has none of the H_RARE flags (MKT, discard, -1 fields), so their
// tests are compiled out of the common FAST add
template <bool G, bool RARE, int S> DEV void bid_lim(Book<S>& B, Msg m) {
    if (!RARE) __builtin_assume(m.qty > 0);  // (decode_msgs: an add of no quantity is RARE)
    constexpr bool POS = !RARE && !G;
    if (POS) {  // the common add: it does not cross (an empty ask side stands for maxint), so all of it goes in
        if (__builtin_expect(B.a.xp > m.price, 1)) {  // (xp: the best ask, an empty side maxint)
            lmask free[S];
            free_slots(B, B.b, free);
            if (!no_slot(free)) {
                add_free<true, false, S, true>(B, B.b, m, m.qty, free);
                return;
            }
            if (B.c.check_fill) evict_if_full<true>(B, B.b, free);
            add_order<true, G>(B, B.b, m, m.qty, free);
            return;
        }
    }
    const i32 rem = match_against<false, G, S, POS>(B, B.a, m.qty, m.price, m);
    if (RARE && __builtin_expect((m.h & H_MKT) != 0, 0)) m.price = B.c.maxint;  // MKT: set after matching (sic)
    lmask free[S];
    free_slots(B, B.b, free);
    if (!no_slot(free)) {
        // FAST: a discarded add is an add of nothing (add_free returns at once for qty <= 0)
        if (!G) add_free<true, RARE>(B, B.b, m, (RARE && (m.h & H_DISCARD)) ? 0 : rem, free);
        else if (!(m.h & H_DISCARD)) add_order<true, G>(B, B.b, m, rem, free);
        return;
    }
    if (B.c.check_fill) evict_if_full<true>(B, B.b, free);
    if (!(m.h & H_DISCARD)) add_order<true, G>(B, B.b, m, rem, free);
}
// ask_lim — :446-508
template <bool G, bool RARE, int S> DEV void ask_lim(Book<S>& B, Msg m) {
    if (!RARE) __builtin_assume(m.qty > 0);  // (decode_msgs: an add of no quantity is RARE)
    if (RARE && __builtin_expect((m.h & H_MKT) != 0, 0)) m.price = 0;
    constexpr bool POS = !RARE && !G;
    if (POS && __builtin_expect(B.b.best_p < m.price, 1)) {  // the common add: it does not cross
        lmask free[S];
        free_slots(B, B.a, free);
        if (!no_slot(free)) {
            add_free<false, false, S, true>(B, B.a, m, m.qty, free);
            return;
        }
        if (B.c.check_fill) evict_if_full<false>(B, B.a, free);
        add_order<false, G>(B, B.a, m, m.qty, free);
        return;
    }
    const i32 rem = match_against<true, G, S, POS>(B, B.b, m.qty, m.price, m);
    lmask free[S];
    free_slots(B, B.a, free);
    if (!no_slot(free)) {
        if (!G) add_free<false, RARE>(B, B.a, m, (RARE && (m.h & H_DISCARD)) ? 0 : rem, free);
        else if (!(m.h & H_DISCARD)) add_order<false, G>(B, B.a, m, rem, free);
        return;
    }
    if (B.c.check_fill) evict_if_full<false>(B, B.a, free);
    if (!(m.h & H_DISCARD)) add_order<false, G>(B, B.a, m, rem, free);
}
// get_random_id_match / get_random_large_id_match — :141-164 (cancel_mode 2/3).
// key = split(key)[0]; chosen = jax.random.choice(key, ids, p=|sign(ids)|),
// ids = the row's order id where `pm` holds, else 0.  choice with p (JAX):
// r = cumsum(p)[-1] * (1 - uniform_f32(key)), ind = searchsorted(cumsum(p), r)
// (side='left').  The weights are 0/1, so the float cumsum is exact and ind is
// the K-th weighted row, K = ceil(r) (ind = 0, chosen = 0, when no row weighs).
// idx = first row whose id == chosen (any row, as jnp.where(ids == chosen)).
template <int S>
DEV int random_id_match(const Book<S>& B, Key& k, const i32 (&o)[S], const lmask (&pm)[S]) {
    k = split_key(k, 2, 0, B.part);
    lmask w[S];
    int tot = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        w[r] = pm[r] & bal(o[r] != 0);
        tot += __builtin_popcountll(w[r]);
    }
    const u32 bits = random_bits(k, 1, 0, B.part);
    const float u = __uint_as_float((bits >> 9) | 0x3f800000u) - 1.0f;
    const float rr = (float)tot * (1.0f - u);
    i32 chosen = 0;
    if (tot > 0) {
        int K = (int)ceilf(rr);
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const int c = __builtin_popcountll(w[r]);
            if (K > 0 && K <= c) {
                const u32 below = __builtin_amdgcn_mbcnt_hi((u32)(w[r] >> 32), __builtin_amdgcn_mbcnt_lo((u32)w[r], 0u));
                const lmask hit = w[r] & bal(below == (u32)(K - 1));
                chosen = rdl(o[r], (int)ff1(hit));
            }
            K -= c;
        }
    }
    lmask f[S];
#pragma unroll
    for (int r = 0; r < S; ++r) f[r] = B.vs.m[r] & bal(o[r] == chosen);
    return first_slot(f, -1);
}
// cancel_order + get_init_id_match — :93-139 (+ :141-164 when RC)
template <bool G, bool ASKS, bool RC, int S> DEV void cancel(Book<S>& B, Side<S>& s, const Msg& m) {
    // On clean sides (the !G variant) a zero-quantity cancel changes nothing: whichever row it
    // picks keeps q (or, empty, stays all -1) and the best quote is unchanged.  The agents'
    // unused cancel rows (getCancelMsgs' zero rows) are such messages.
    if (!G && m.qty == 0) return;
    const int R = B.c.nO;
    i32 o[S], q[S];
    ldcol(s.t, R, FOID, o);
    ldcol(s.t, R, FQ, q);
    lmask fm[S];
#pragma unroll
    for (int r = 0; r < S; ++r) fm[r] = B.vs.m[r] & bal(o[r] == m.oid);
    int idx = first_slot(fm, -1);
    if (idx < 0) {
        // get_init_id_match: price == msg price, init_id - 2 * depth <= oid <= init_id, q >= msg q.
        // Evaluated per lane in VALU (selects feeding one compare), not as three lane masks ANDed on
        // the scalar unit: oid in range <=> (u32)(oid - lo) <= (u32)(init_id - lo), given lo <= init_id
        // (check_lob refuses book_depth < 0 and an overflowing init_id - 2 * book_depth).
        const i32 lo = wsub(B.c.init_id, wmul(B.c.depth, 2));
        const u32 span = (u32)wsub(B.c.init_id, lo);
#pragma unroll
        for (int r = 0; r < S; ++r) {
            u32 d = vkeep((u32)wsub(o[r], lo));
            d = vkeep(s.pc[r] == m.price ? d : 0xFFFFFFFFu);
            d = vkeep(q[r] >= m.qty ? d : 0xFFFFFFFFu);
            fm[r] = B.vs.m[r] & bal(d <= span);
        }
        if (!RC) {
            idx = first_slot(fm, R - 1);  // -1 wraps to the last slot
        } else {
            idx = first_slot(fm, -1);
            if (idx < 0 && B.c.cancel_mode >= 2) {
                Key k = split_key(B.ek, B.nmsg, B.mi, B.part);
#pragma unroll
                for (int r = 0; r < S; ++r) fm[r] = B.vs.m[r] & bal(s.pc[r] == m.price) & bal(q[r] >= m.qty);
                idx = random_id_match(B, k, o, fm);
                if (idx < 0 && B.c.cancel_mode == 3) {
#pragma unroll
                    for (int r = 0; r < S; ++r) fm[r] = B.vs.m[r] & bal(s.pc[r] == m.price);
                    idx = random_id_match(B, k, o, fm);
                }
            }
            if (idx < 0) idx = R - 1;
        }
    }
    const i32 op = sget(s.pc, idx), oq = sget(q, idx);
    // FAST sides: a p == -1 row holds -1 in every field but q (a cancel of a negative quantity can
    // leave q > 0 there).  Cancelling qty >= -1 from an all -1 row leaves q = -1 - qty <= 0, which
    // _removeZeroNegQuant clears back to all -1: the book and its best quotes are unchanged.  This
    // is the common cancel of the replayed data (an order id the episode's book does not hold, no
    // init-id match: the -1 index wraps to the last slot, usually empty; tools/msg_mix.py).
    // (two plain branches: as one condition the compiler ANDs two 64-bit lane masks on the scalar
    // unit, 8 instructions instead of 3 / 5)
    if (!G && fresh(op & oq) == -1) {
        asm volatile("");
        if (m.qty >= -1) return;
    }
    const i32 nq = wsub(oq, m.qty);
    if (!G || (B.fl & SideBits<ASKS>::CLEAN)) {
        if (nq <= 0) side_clr(s, R, idx);
        else stu(s.t, s.scr, R, FQ, idx, nq);
        note_reduce<ASKS>(s, B.fl, op, wsub(oq, nq > 0 ? nq : 0), m.k);
    } else {
        stu(s.t, s.scr, R, FQ, idx, nq);
        rzn<ASKS>(s, B.fl, R, B.vs);
    }
}

// cond_type_side_save_bidask — :687-732: dispatch index
//   1 side==1 & type in {1,4}; 2 side==-1 & type in {2,3}; 3 side==1 & type in {2,3};
//   4 side==0 & type==0 (doNothing); everything else 0 (ask_lim); side flipped for type 4.
// Evaluated in VALU for the 64 messages of a chunk at once (lane = message):
// x = (type, side, qty, price) becomes (handler | flags, side', qty, price).
// H_DISCARD: a type-4 message under type_4_interpretation 0/2 is not added
// after matching.  H_NEG1: the row add_order would write has p != -1 and a -1
// in another field (it sets the side's NEG1 flag); the price it writes is the
// message's, or maxint / 0 for MKT bids / asks.  H_PM1: that price is -1 (the
// row would be an order priced -1: the side's PM1 flag).
DEV void decode_msgs(const LobCfg& c, int4& x, const int4& y) {
    const i32 ty = x.x, sd = ty == 4 ? wsub(0, x.y) : x.y;
    const bool cnl = (ty == 2) | (ty == 3);
    i32 h = H_ASK;
    h = (((ty == 0) & (sd == 0))) ? H_NOP : h;
    h = (((ty == 1) | (ty == 4)) & (sd == 1)) ? H_BID : h;
    h = (cnl & (sd == 1)) ? H_CNL_BID : h;
    h = (cnl & (sd == -1)) ? H_CNL_ASK : h;
    if (((c.t4 == 0) | (c.t4 == 2)) & (ty == 4)) h |= H_DISCARD;
    const i32 p_add = c.t4 == 2 ? (h == H_BID ? c.maxint : 0) : x.w;
    if ((p_add != -1) & ((y.x == -1) | (y.y == -1) | (y.z == -1) | (y.w == -1))) h |= H_NEG1;
    if (p_add == -1) h |= H_PM1;  // an add would write an order priced -1
    if (c.t4 == 2) h |= H_MKT;    // type_4_interpretation MKT: the limit handlers' price overrides
    if (h & (H_DISCARD | H_NEG1 | H_PM1 | H_MKT)) h |= H_RARE;
    if ((h <= H_BID) & (x.z <= 0)) h |= H_RARE;  // an add of no quantity (the common add handlers assume qty > 0)
    if (((h & H_KIND) == H_ASK) & (sd != -1)) h |= H_RARE;  // (a common bid has side 1, a common ask -1)
    if ((h <= H_BID) & (x.w < 0)) h |= H_RARE;  // a negative price (the common adds' note_add assumes p >= 0)
    x.x = h;
    x.y = sd;
}
// sdv: the chunk's side register (decode_msgs), read at lane k only where a handler needs the
// side: a common (not RARE) bid has side 1 and a common ask -1, and only matches record it
template <bool G, bool RC, int S>
DEV void process_msg_(Book<S>& B, u32 k, i32 h, i32 sdv, i32 d2, i32 d3, i32 d4, i32 d5, i32 d6, i32 d7) {
    Msg m;
    m.h = h; m.side = 0; m.price = d3; m.qty = d2; m.oid = d4; m.tid = d5; m.t = d6; m.tns = d7;
    m.k = k;
    const i32 kind = h & H_KIND;
    if (kind == H_CNL_ASK) cancel<G, true, RC>(B, B.a, m);
    else if (kind == H_CNL_BID) cancel<G, false, RC>(B, B.b, m);
    else if (kind == H_BID) {
        if (!G && !(h & H_RARE)) {
            m.side = 1;
            bid_lim<G, false>(B, m);
        } else {
            m.side = rdl(sdv, k);
            bid_lim<G, true>(B, m);
        }
    } else if (kind == H_ASK) {
        if (!G && !(h & H_RARE)) {
            m.side = -1;
            ask_lim<G, false>(B, m);
        } else {
            m.side = rdl(sdv, k);
            ask_lim<G, true>(B, m);
        }
    }
}

// forward fill of -1 prices across the lanes of a chunk (carry = last price before it)
DEV i32 ffill(i32 v, i32 carry) {
    const int l = lane_id();
    const lmask m = bal(v != -1) & (~0ull >> (63 - l));  // lanes <= l holding a price
    const int src = m ? 63 - __builtin_clzll(m) : -1;
    const i32 got = __builtin_amdgcn_ds_bpermute(src << 2, v);
    return src < 0 ? carry : got;
}
// REC: after message k (which records the recomputed quotes), not at a chunk's start
template <bool REC = true, int S> DEV void refresh_best(Book<S>& B, u32 k = 0) {
    if (B.fl & STALE_ANY) {
        if (B.fl & F_STALE_A) rescan<true, REC>(B.a, B.fl, B.c.nO, B.vs, B.c.maxint, k);
        if (B.fl & F_STALE_B) rescan<false, REC>(B.b, B.fl, B.c.nO, B.vs, B.c.maxint, k);
        B.fl &= ~STALE_ANY;
    }
}

// ------------------------------------------------- chunk pre-pass: no-op messages
// Which of a chunk's messages provably leave the book as it is, decided for the 64 messages at
// once in VALU before the serial loop; the loop skips them and their best-quote record is the
// previous message's (the book, hence get_best_* and get_volume_at_price, is unchanged).
//  - doNothing rows (cond_type_side index 4: no branch of the lax.switch writes anything);
//  - on a FAST book (both sides clean, no -1 oddities, the kernels' common variant) and before
//    the first message that can end it: a cancel of quantity 0 (cancel_order subtracts 0 from
//    whichever row it picks, JaxOrderBookArrays.py:93-139), and the replayed day's common cancel
//    (DESIGN.md §4): an order id no row holds, no get_init_id_match candidate at its price, so
//    the -1 index wraps to the last slot (:132-139) which is an all -1 row and stays one until
//    the message (fewer adds to that side before it than free rows below the last slot, and only
//    adds fill rows), and a quantity >= -1: q = -1 - qty <= 0 and _removeZeroNegQuant (:85-90)
//    restores the all -1 row.
// "No row holds the id / no candidate at the price" is a one-hash Bloom filter over the book's
// ids and init-id rows' (price, side) at chunk start plus the chunk's add ids: a false positive
// only means the message runs.  A message that can end the FAST variant or create a candidate
// (an add with a -1 field, priced -1 or carrying an init id; a cancel of a negative quantity,
// which can leave q > 0 in an empty row) ends the skipping for the rest of the chunk.
DEV u32 hash_id(i32 v) { return ((u32)v * 0x9E3779B1u) >> 21; }
DEV u32 hash_px(i32 p, bool ask) { return (((u32)p * 0x85EBCA6Bu) ^ (ask ? 0xC2B2AE35u : 0x27D4EB2Fu)) >> 21; }
DEV void filt_set(i32* f, u32 h, bool on) {
    __hip_atomic_fetch_or(reinterpret_cast<u32*>(f) + (h >> 5), on ? 1u << (h & 31) : 0u, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
}
DEV u32 filt_get(const i32* f, u32 h) { return ((u32)f[h >> 5] >> (h & 31)) & 1u; }
DEV u32 lanes_below(lmask m) { return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u)); }
// -1 if the side's last slot is not an all -1 row, else the number of p == -1 rows below it
template <int S> DEV int side_room(const Book<S>& B, const Side<S>& s) {
    const int R = B.c.nO, rl = (R - 1) >> 6, ll = (R - 1) & 63;
    int n = 0;
    bool last = false;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        lmask f = B.vs.m[r] & bal(s.pc[r] == -1);
        if (r == rl) {
            last = (f >> ll) & 1ull;
            f &= ~(1ull << ll);
        }
        n += __builtin_popcountll(f);
    }
    if (!last) return -1;
    return ldu(s.t, R, FQ, R - 1) == -1 ? n : -1;
}
// x, y: the chunk's decoded messages (decode_msgs), lane = message; cnt: messages in the chunk
template <bool RC, int S> DEV lmask chunk_noops(Book<S>& B, const int4& x, const int4& y, int cnt) {
    const int l = lane_id();
    const i32 kind = x.x & H_KIND, qty = x.z, price = x.w, oid = y.x;
    const bool in = l < cnt;
    const lmask nop = bal(in & (kind == H_NOP));
    if ((i32)B.fl < 0) {  // not FAST (F_SLOW)
        B.filt_ok = false;
        return nop;
    }
    const bool cnl = (kind == H_CNL_ASK) | (kind == H_CNL_BID), add = (kind == H_ASK) | (kind == H_BID);
    const i32 lo = wsub(B.c.init_id, wmul(B.c.depth, 2));
    const u32 span = (u32)wsub(B.c.init_id, lo);
    const bool init_oid = (u32)wsub(oid, lo) <= span;
    const lmask brk = bal(in & ((add & (((x.x & (H_NEG1 | H_PM1)) != 0) | init_oid)) | (cnl & (qty < -1))));
    const lmask before = brk ? (1ull << ff1(brk)) - 1ull : ~0ull;
    const lmask zero = bal(in & cnl & (qty == 0)) & before;
    if (RC || (u32)wsub(-1, lo) <= span) return nop | zero;  // (-1 ids would be init-id candidates)
    i32* f = B.filt;
    if (!B.filt_ok) {  // the book's ids and init-id rows' (price, side), as they are now
        f[l] = 0;
        wave_sync();
        const int R = B.c.nO;
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
            const Side<S>& s = sd ? B.b : B.a;
            i32 o[S];
            ldcol(s.t, R, FOID, o);
#pragma unroll
            for (int r = 0; r < S; ++r) {
                filt_set(f, hash_id(o[r]), B.vs.v[r] & (o[r] != -1));
                filt_set(f, hash_px(s.pc[r], sd == 0), B.vs.v[r] & ((u32)wsub(o[r], lo) <= span));
            }
        }
    }
    // the chunk's add ids.  Only adds write rows (their ids go in here), a row's price never changes and
    // init-id rows come from nowhere else than an add carrying an init id (a brk message), so without a
    // brk message the filter stays a superset of the book's ids and init rows for the next chunk
    filt_set(f, hash_id(oid), in & add);
    B.filt_ok = brk == 0ull;
    wave_sync();
    const bool ask = kind == H_CNL_ASK;
    const bool hit = (filt_get(f, hash_id(oid)) | filt_get(f, hash_px(price, ask))) != 0u;
    const int room_a = side_room(B, B.a), room_b = side_room(B, B.b);
    const u32 adds_a = lanes_below(bal(in & (kind == H_ASK))), adds_b = lanes_below(bal(in & (kind == H_BID)));
    const int room = ask ? room_a : room_b;
    const i32 adds = (i32)(ask ? adds_a : adds_b);
    const bool quiet = in & cnl & (qty >= -1) & (oid != -1) & !hit & (room >= 0) & (adds <= room);
    return nop | zero | (bal(quiet) & before);
}

// One chunk of the message scan: the chunk's messages that are not no-ops (chunk_noops) through
// the book in order, each followed by its best-quote record (lane k of rpa / rqa / rpb / rqb:
// get_best_ask / its volume, get_best_bid / its volume after message k); a skipped message
// records the quotes after the message before it.  base: the chunk's first message index.
template <bool RC, int S>
DEV void run_chunk(Book<S>& B, const int4& x, const int4& y, int cnt, int base, i32& rpa, i32& rqa, i32& rpb,
                   i32& rqb) {
    const lmask live = cnt >= 64 ? ~0ull : (1ull << cnt) - 1ull;
#ifdef HFTLOB_NO_SKIP  // A/B builds only
    const lmask skip = 0;
#else
    const lmask skip = chunk_noops<RC>(B, x, y, cnt) & live;
#endif
    lmask todo = live & ~skip;
#ifdef HFTLOB_KO_LOOP  // timing knockout builds only (wrong results): no message reaches the book
    todo = 0;
#endif
    refresh_best<false>(B);
    const i32 cpa = B.a.best_p, cqa = B.a.best_q, cpb = B.b.best_p, cqb = B.b.best_q;  // before the chunk
    // the best-quote record: a message that sets or recomputes a side's quote writes it into its
    // lane of that side's record (side_rec, at the assignment); the other lanes take the last
    // record before them below (the book, hence that quote, is unchanged since)
    B.a.rm = B.b.rm = 0ull;
    B.a.rp = B.a.rq = B.b.rp = B.b.rq = 0;
    if (todo) {
        // message k's fields are read (v_readlane) at the end of the message before it, so their
        // latency overlaps the best-quote record and the loop test instead of stalling the dispatch
        u32 k = ff1(todo);
        i32 h = rdl(x.x, k), d2 = rdl(x.z, k), d3 = rdl(x.w, k), d4 = rdl(y.x, k),
            d5 = rdl(y.y, k), d6 = rdl(y.z, k), d7 = rdl(y.w, k);
        do {
            asm volatile("s_bitset0_b64 %0, %1" : "+s"(todo) : "s"(k));
            if (RC) B.mi = base + (int)k;
            if ((i32)B.fl >= 0) process_msg_<false, RC>(B, k, h, x.y, d2, d3, d4, d5, d6, d7);  // (!F_SLOW)
            else process_msg_<true, RC>(B, k, h, x.y, d2, d3, d4, d5, d6, d7);
            refresh_best(B, k);
            const u32 kn = ff1(todo);  // (-1 once todo is empty: v_readlane takes the lane's low 6 bits)
            h = rdl(x.x, kn); d2 = rdl(x.z, kn); d3 = rdl(x.w, kn);
            d4 = rdl(y.x, kn); d5 = rdl(y.y, kn); d6 = rdl(y.z, kn); d7 = rdl(y.w, kn);
            k = kn;
        } while (todo);
    }
    {  // every lane takes its side's last record at or before it (or the chunk's starting quote)
        const int l = lane_id();
        const lmask below = ~0ull >> (63 - l);
        const lmask ma = B.a.rm & below, mb = B.b.rm & below;
        const int sa = ma ? 63 - __builtin_clzll(ma) : -1, sb = mb ? 63 - __builtin_clzll(mb) : -1;
        const i32 gpa = __builtin_amdgcn_ds_bpermute(sa << 2, B.a.rp), gqa = __builtin_amdgcn_ds_bpermute(sa << 2, B.a.rq);
        const i32 gpb = __builtin_amdgcn_ds_bpermute(sb << 2, B.b.rp), gqb = __builtin_amdgcn_ds_bpermute(sb << 2, B.b.rq);
        rpa = sa < 0 ? cpa : gpa;
        rqa = sa < 0 ? cqa : gqa;
        rpb = sb < 0 ? cpb : gpb;
        rqb = sb < 0 ? cqb : gqb;
    }
}

// LDS carve-up of one env's book: [asks 6*nO][bids 6*nO][trades 8*nT][pad 64*4]
// (column loads read past the trades (lanes masked by Valid; up to 127 words at the 100/100
// sizes): the first 128 pad words; then the chunk_noops filter (64 words) and the store scratch
// row (64 words), which over-reads at small nT may also read)
template <int S> DEV void book_bind(Book<S>& B, i32* lds) {
    B.a.t = lds;
    B.b.t = lds + 6 * B.c.nO;
    B.tr.t = lds + 12 * B.c.nO;
    B.tr.R = B.c.nT;
    B.filt = lds + 12 * B.c.nO + 8 * B.c.nT + 128;
    B.filt_ok = false;
    B.a.scr = B.b.scr = B.tr.scr = lds + 12 * B.c.nO + 8 * B.c.nT + 192;
    B.vs.init(B.c.nO);
    B.vt.init(B.c.nT);
}

// ================================================= K1: book_process kernel
// scan_through_entire_array[_save_bidask] — JaxOrderBookArrays.py:736-823
// RC: cancel_mode 2/3 (keys[e] is the scan's key; message k uses split(key, n_msg)[k])
template <int S, bool RC>
__global__ __launch_bounds__(64) void k_book_process(hftlob_lob_cfg cfg, int n_env, int n_msg, const u32* __restrict__ keys,
                                                     const i32* __restrict__ msgs,
                                                     i32* __restrict__ asks, i32* __restrict__ bids,
                                                     i32* __restrict__ trades, i32* __restrict__ best_asks,
                                                     i32* __restrict__ best_bids) {
    one_wave();
    extern __shared__ __attribute__((aligned(16))) i32 lds[];
    const int e = blockIdx.x;
    if (e >= n_env) return;
    const int l = lane_id();
    Book<S> B;
    B.c = lobcfg(cfg);
    book_bind(B, lds);
    const int R = B.c.nO;
    i32* ga = asks + (size_t)e * R * 6;
    i32* gb = bids + (size_t)e * R * 6;
    i32* gt = trades + (size_t)e * B.c.nT * 8;
    B.fl = load_side<true>(B.a, ga, R, B.vs) | load_side<false>(B.b, gb, R, B.vs) | F_STALE_A | F_STALE_B | STALE_ANY;
    B.fl |= slow_bit(B.fl);
    load_trades(B.tr, gt, B.vt);
    {  // the loaded log's free-row prefix (see Book::ntr)
        lmask fr[S], bad = 0;
#pragma unroll
        for (int r = 0; r < S; ++r) fr[r] = B.vt.m[r] & bal(B.tr.get(4, r) == -1);
        const int first = first_slot(fr, B.c.nT);
        const int l = lane_id();
#pragma unroll
        for (int r = 0; r < S; ++r) bad |= B.vt.m[r] & ~fr[r] & bal(r * 64 + l >= first);
        B.ntr = bad == 0ull ? first : -1;
    }
    if (RC) {
        B.ek = Key{keys[2 * e], keys[2 * e + 1]};
        B.nmsg = n_msg;
        B.part = cfg.prng_partitionable;
    }
    const i32* gm = msgs + (size_t)e * n_msg * 8;
    int4 nx = make_int4(0, 0, 0, 0), ny = nx;  // message rows, loaded one chunk ahead
    if (l < n_msg) {
        nx = reinterpret_cast<const int4*>(gm + l * 8)[0];
        ny = reinterpret_cast<const int4*>(gm + l * 8)[1];
    }
    for (int base = 0; base < n_msg; base += 64) {
        const int row = base + l;
        int4 x = nx, y = ny;
        nx = make_int4(0, 0, 0, 0);
        ny = nx;
        if (row + 64 < n_msg) {  // the next chunk's loads land while this one runs
            nx = reinterpret_cast<const int4*>(gm + (row + 64) * 8)[0];
            ny = reinterpret_cast<const int4*>(gm + (row + 64) * 8)[1];
        }
        decode_msgs(B.c, x, y);
        i32 ap = 0, aq = 0, bp = 0, bq = 0;
        const int cnt = uni(imin_(64, n_msg - base));  // SGPR: the loop test stays on the scalar unit
        run_chunk<RC>(B, x, y, cnt, base, ap, aq, bp, bq);
        if (best_asks && row < n_msg) {
            reinterpret_cast<int2*>(best_asks + ((size_t)e * n_msg + row) * 2)[0] = make_int2(ap, aq);
            reinterpret_cast<int2*>(best_bids + ((size_t)e * n_msg + row) * 2)[0] = make_int2(bp, bq);
        }
    }
    store_side(B.a, ga, R, B.vs);
    store_side(B.b, gb, R, B.vs);
    store_trades(B.tr, gt, B.vt);
}

// =========================================================== env helpers
struct EnvCfg {
    const hftlob_env_cfg* c;
};

// world/loaded word indices inside the record (hftlob.h)
enum { LD_T0 = 0, LD_T1, LD_WIN, LD_MAXS, LD_START, LD_STEP };
enum { W_T0 = 0, W_T1, W_OIDC, W_MID, W_DT };

DEV int agent_words(const hftlob_agent_type_cfg& t) { return t.kind == HFTLOB_AGENT_MM ? 5 : 13; }

// side volume (get_volume — :919-930)
template <int S> DEV i32 side_volume_pq(const i32 (&p)[S], const i32 (&q)[S], const Valid<S>& V) {
    i32 v = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) v = wadd(v, (V.v[r] && p[r] != -1) ? q[r] : 0);
    return wave_sum(v);
}
template <int S> DEV i32 side_volume(const Side<S>& s, int R, const Valid<S>& V) {
    i32 q[S];
    ldcol(s.t, R, FQ, q);
    return side_volume_pq(s.pc, q, V);
}
// prices and quantities of a global [R][6] side, lane-strided into registers
template <int S> DEV void global_pq(const i32* g, const Valid<S>& V, i32 (&p)[S], i32 (&q)[S]) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        p[r] = q[r] = -1;
        if (V.v[r]) {
            const int2 x = reinterpret_cast<const int2*>(g + (r * 64 + l) * 6)[0];
            p[r] = x.x; q[r] = x.y;
        }
    }
}

// canonical float sum of per-row values over n rows held S-strided
// Independent scalar float divisions of one agent's reward, evaluated together: division k's
// operands in lane k, one vector division, results read back per lane (the same IEEE quotients as
// k separate scalar divisions, with one division's latency instead of k in a chain)
struct DivBatch {
    int l;
    float n = 0.0f, d = 1.0f, q = 0.0f;
    DEV void add(int k, float num, float den) {
        n = l == k ? num : n;
        d = l == k ? den : d;
    }
    DEV void run() { q = n / d; }
    DEV float get(int k) const { return unif_lane(q, k); }
    DEV static float unif_lane(float v, int k) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k)); }
};
// rows_fsum of n rows that all hold the same signed zero z: z when every lane sums rows (n >= 64),
// +0 otherwise (the lanes past n add +0)
DEV float zsum(float z, int n) { return n >= 64 ? z : z + 0.0f; }
template <int S> DEV float rows_fsum(const float (&x)[S], int n) {
    const int l = lane_id();
    float a = l < n ? x[0] : 0.0f;
#pragma unroll
    for (int r = 1; r < S; ++r) if (r * 64 + l < n) a = a + x[r];
    return wave_fsum(a);
}

// One agent's observation row, one field per lane: put(k, x, off, div) keeps field k's raw value x
// and its normalisation (x - off) / div (normalize_obs, mm_env.py:3157-3167: (x - mean) / std) in
// lane k, and fin() divides once for all fields (one vector division instead of one per field;
// the same IEEE operations per field: x - 0 == x and x / 1 == x exactly).  (The obs functions
// fill fields by config-dependent branches; a local float array written that way ends up in
// scratch memory, with a scratch store per field per lane.)
struct ObsLane {
    int l;
    float v = 0.0f, off = 0.0f, div = 1.0f;
    DEV void put(int k, float x, float o, float d) {
        const bool me = l == k;
        v = me ? x : v;
        off = me ? o : off;
        div = me ? d : div;
    }
    DEV void put_i(int k, i32 x) { v = l == k ? __int_as_float(x) : v; }  // an int32 field, kept as its bits
    DEV float fin() const { return (v - off) / div; }
};

struct WorldView {  // wave-uniform world quantities used by obs
    i32 best_ask_p, best_bid_p, vol_a, vol_b, step, max_steps;
    float mid;
    // fixed_time episodes (EXE engineered obs): world time, init_time, delta_time
    i32 t0, t1, it0, it1;
    float dt;
};

// MM _get_obs_basic / _get_obs_engineered, sorted keys — mm_env.py:2963-3154.
// RAW: get_observation(normalize=False, flatten=False) for save_raw_observations
// (marl_env.py:684-685): no normalisation, and the int32 fields keep their int32
// value (stored as int bits; flattening is what casts them to float).
// OBS_F: a float field x, normalised (x - o) / d; OBS_I: an int32 field x, as float i2f(x)
#define OBS_F(k, x, o_, d_) o.put((k), (x), nz ? (o_) : 0.0f, nz ? (d_) : 1.0f)
#define OBS_I(k, x, o_, d_) do { if (RAW) o.put_i((k), (x)); else OBS_F((k), i2f(x), (o_), (d_)); } while (0)
template <bool RAW>
DEV void mm_obs(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, const WorldView& w, const i32* st, ObsLane& o,
                bool ftime) {
    const bool nz = !RAW && tc.normalize;
    const i32 spread = iabs_(wsub(w.best_ask_p, w.best_bid_p));
    if (tc.observation_space == HFTLOB_MM_OBS_BASIC) {  // inventory, spread
        OBS_I(0, st[2], 0.0f, 10.0f);
        OBS_I(1, spread, 0.0f, 1e4f);
        return;
    }
    // "messages" (mm_env.py:2820-2821): the observation is the step's message array, written
    // by env_step_dev to out.msgs; the float row stays zero
    if (tc.observation_space == HFTLOB_MM_OBS_MESSAGES) return;
    if (ftime) {  // mm_env.py:3029-3088, sorted keys: delta_time, inventory, mid_price, p_ask, p_bid, q_ask,
                  // q_bid, spread, step_counter, time_remaining
        const float tm = i2f(w.t0) + i2f(w.t1) / 1e9f;
        const float trem = (float)c.episode_time - (tm - (i2f(w.it0) + i2f(w.it1) / 1e9f));
        OBS_F(0, w.dt, 0.0f, 10.0f);
        OBS_I(1, st[2], 0.0f, 10.0f);
        OBS_F(2, w.mid, 0.0f, 1e6f);
        OBS_I(3, w.best_ask_p, 0.0f, 1e6f);
        OBS_I(4, w.best_bid_p, 0.0f, 1e6f);
        OBS_I(5, w.vol_a, 0.0f, 1000.0f);
        OBS_I(6, w.vol_b, 0.0f, 1000.0f);
        OBS_I(7, spread, 0.0f, 1e4f);
        OBS_I(8, w.step, 0.0f, 10.0f);
        OBS_F(9, trem, 0.0f, (float)c.episode_time);
        return;
    }
    // fixed_steps: inventory, mid_price, p_ask, p_bid, q_ask, q_bid, spread, step_counter
    OBS_I(0, st[2], 0.0f, 10.0f);
    OBS_F(1, w.mid, 0.0f, 1e6f);
    OBS_I(2, w.best_ask_p, 0.0f, 1e6f);
    OBS_I(3, w.best_bid_p, 0.0f, 1e6f);
    OBS_I(4, w.vol_a, 0.0f, 1000.0f);
    OBS_I(5, w.vol_b, 0.0f, 1000.0f);
    OBS_I(6, spread, 0.0f, 1e4f);
    OBS_I(7, w.step, 0.0f, 10.0f);
}
// EXE _get_obs / _get_obs_basic / _get_obs_simplest_case, sorted keys — exec_env.py:1841-2079
// ftime: ep_type == fixed_time, passed by the caller (compile-time false in the 100/100 kernel)
template <bool RAW>
DEV void exe_obs(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, const WorldView& w, const i32* st, ObsLane& o,
                 bool ftime) {
    const bool nz = !RAW && tc.normalize;
    if (tc.observation_space == HFTLOB_EXE_OBS_BASIC) {  // :1879-1911 best_ask_price, best_bid_price, remaining_quant
        // (normalised: the int32 price minus 1550000, then / 1e3)
        const i32 rq = wsub(st[1], st[2]);
        if (RAW) {
            o.put_i(0, w.best_ask_p);
            o.put_i(1, w.best_bid_p);
        } else {
            o.put(0, i2f(nz ? wsub(w.best_ask_p, 1550000) : w.best_ask_p), 0.0f, nz ? 1e3f : 1.0f);
            o.put(1, i2f(nz ? wsub(w.best_bid_p, 1550000) : w.best_bid_p), 0.0f, nz ? 1e3f : 1.0f);
        }
        OBS_I(2, rq, 0.0f, (float)tc.task_size);
        return;
    }
    if (tc.observation_space == HFTLOB_EXE_OBS_SIMPLEST_CASE) {
        // :1841-1877 mid_price, percent_remaining_quant, percent_time_remaining (all float32)
        const float ep = (float)c.episode_time;
        const float ptr = (ep - (i2f(wsub(w.t0, w.it0)) + i2f(wsub(w.t1, w.it1)) / 1e9f)) / ep;
        const float prq = i2f(wsub(st[1], st[2])) / i2f(st[1]);
        OBS_F(0, w.mid, 7560000.0f, 1e3f);
        OBS_F(1, prq, 0.5f, 1.0f);
        OBS_F(2, ptr, 0.5f, 1.0f);
        return;
    }
    const i32 sell = st[3];
    const i32 p_aggr = sell ? w.best_bid_p : w.best_ask_p, p_pass = sell ? w.best_ask_p : w.best_bid_p;
    const i32 q_aggr = sell ? w.vol_b : w.vol_a, q_pass = sell ? w.vol_a : w.vol_b;
    const float ip = bitf(st[0]);
    const float ts = (float)tc.task_size;
    const float rr = w.max_steps == 0 ? 0.0f : 1.0f - i2f(w.step) / i2f(w.max_steps);
    const i32 spr = iabs_(wsub(p_aggr, p_pass)), rq = wsub(st[1], st[2]);
    int k = 0;
    if (ftime) {
        // fixed_time (exec_env.py:1940-2010): 15 keys, sorted: delta_time, executed_quant, init_price,
        // is_sell_task, p_aggr, p_pass, q_aggr, q_pass, remaining_quant, remaining_ratio, spread,
        // step_counter, task_size, time, time_remaining
        OBS_F(0, w.dt, 0.0f, 10.0f);
        k = 1;
    }
    // fixed_steps (12 keys): executed_quant, init_price, is_sell_task, p_aggr, p_pass, q_aggr, q_pass,
    // remaining_quant, remaining_ratio, spread, step_counter, task_size
    OBS_I(k + 0, st[2], 0.0f, ts);
    OBS_F(k + 1, ip, 0.0f, 1e7f);
    OBS_I(k + 2, sell, 0.0f, 1.0f);
    OBS_I(k + 3, p_aggr, ip, 1e5f);
    OBS_I(k + 4, p_pass, ip, 1e5f);
    OBS_I(k + 5, q_aggr, 0.0f, 1000.0f);
    OBS_I(k + 6, q_pass, 0.0f, 1000.0f);
    OBS_I(k + 7, rq, 0.0f, ts);
    OBS_F(k + 8, rr, 0.0f, 1.0f);
    OBS_I(k + 9, spr, 0.0f, 1e4f);
    OBS_I(k + 10, w.step, 0.0f, 30.0f);
    OBS_I(k + 11, st[1], 0.0f, ts);
    if (ftime) {
        const float tm = i2f(w.t0) + i2f(w.t1) / 1e9f;
        const float trem = (float)c.episode_time - (tm - (i2f(w.it0) + i2f(w.it1) / 1e9f));
        OBS_F(13, tm, 0.0f, 1e5f);
        OBS_F(14, trem, 0.0f, (float)c.episode_time);
    }
}
#undef OBS_I
#undef OBS_F
// write one agent's obs row (lanes 0..obs_stride-1 store one 32-bit word each);
// RAW: the un-normalised row of obs_raw
template <bool RAW>
DEV void write_obs(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, const WorldView& w, const i32* st,
                   void* dst, bool zero, bool ftime) {
    const int l = lane_id();
    ObsLane o{l};
    if (tc.kind == HFTLOB_AGENT_MM) mm_obs<RAW>(c, tc, w, st, o, ftime);
    else exe_obs<RAW>(c, tc, w, st, o, ftime);
    const float v = zero ? 0.0f : (RAW ? o.v : o.fin());
    if (l < c.obs_stride) static_cast<float*>(dst)[l] = v;
}

// ----------------------------------------- reset (MARLEnv.reset_env) device
// marl_env.py:129-207; BaseLOBEnv.reset_env base_env.py:218-234; agents
// mm_env.py:417-459, exec_env.py:209-266.  Writes the whole record + obs.
template <int S>
DEV void env_reset_dev(const hftlob_env_cfg& c, Key key, const i32* __restrict__ init_states, i32* __restrict__ rec,
                       float* __restrict__ obs, const Valid<S>& VS, const Valid<S>& VT, bool ftime) {
    const bool part = c.prng_partitionable;
    const int nTy = c.n_types, l = lane_id();
    Key wk = split_key(key, nTy + 1, nTy, part);
    i32 idx = c.window_selector == -1 ? randint(wk, 0, c.n_windows, part) : c.window_selector;
    idx = imin_(imax_(idx, 0), c.n_windows - 1);
    const i32* src = init_states + (size_t)idx * c.init_rec_words;
    // copy the LoadedEnvState prefix (asks, bids, trades, 6 scalars), 16B vectors
    for (int w = l * 4; w < c.init_rec_words; w += 256) {
        if (w + 3 < c.init_rec_words) {
            *reinterpret_cast<int4*>(rec + w) = *reinterpret_cast<const int4*>(src + w);
        } else {
            for (int k = w; k < c.init_rec_words; ++k) rec[k] = src[k];
        }
    }
    i32 ap[S], aq[S], bp[S], bq[S], ba_p, ba_q, bb_p, bb_q;
    global_pq(src + c.off_asks, VS, ap, aq);
    global_pq(src + c.off_bids, VS, bp, bq);
    best_ask_pq(ap, aq, VS, c.lob.maxint, ba_p, ba_q);
    best_bid_pq(bp, bq, VS, bb_p, bb_q);
    // tile best quotes over M rows
    for (int m = l; m < c.n_msgs; m += 64) {
        reinterpret_cast<int2*>(rec + c.off_best_asks)[m] = make_int2(ba_p, ba_q);
        reinterpret_cast<int2*>(rec + c.off_best_bids)[m] = make_int2(bb_p, bb_q);
    }
    const float mid = i2f(wadd(bb_p, ba_p)) / 2.0f;
    const i32 t0 = src[c.off_loaded + LD_T0], t1 = src[c.off_loaded + LD_T1];
    if (l == 0) {
        i32* W = rec + c.off_world;
        W[W_T0] = t0; W[W_T1] = t1; W[W_OIDC] = c.order_id_counter_start; W[W_MID] = fbit(mid); W[W_DT] = fbit(0.0f);
    }
    WorldView wv;
    wv.best_ask_p = ba_p; wv.best_bid_p = bb_p;
    wv.vol_a = side_volume_pq(ap, aq, VS); wv.vol_b = side_volume_pq(bp, bq, VS);
    wv.step = src[c.off_loaded + LD_STEP]; wv.max_steps = src[c.off_loaded + LD_MAXS]; wv.mid = mid;
    wv.t0 = wv.it0 = t0; wv.t1 = wv.it1 = t1; wv.dt = 0.0f;  // world time = init_time, delta_time 0
    // zero the record's padding words (after the world block, after the agents)
    int agents_end = c.off_agents;
    for (int t = 0; t < nTy; ++t) agents_end += c.types[t].n_agents * agent_words(c.types[t]);
    for (int w = c.off_world + 5 + l; w < c.off_agents; w += 64) rec[w] = 0;
    for (int w = agents_end + l; w < c.rec_words; w += 64) rec[w] = 0;
    i32* st = rec + c.off_agents;
    int ag = 0;
    for (int t = 0; t < nTy; ++t) {
        const hftlob_agent_type_cfg& tc = c.types[t];
        i32 sell = tc.task == HFTLOB_TASK_SELL ? 1 : 0;
        if (tc.kind == HFTLOB_AGENT_EXE && tc.task == HFTLOB_TASK_RANDOM)
            sell = randint(split_key(key, nTy + 1, t, part), 0, 2, part);
        for (int i = 0; i < tc.n_agents; ++i, ++ag) {
            i32 s[13];
            if (tc.kind == HFTLOB_AGENT_MM) {
                s[0] = 0; s[1] = 0; s[2] = 0; s[3] = fbit(0.0f); s[4] = fbit(0.0f);
            } else {
                s[0] = fbit(mid); s[1] = tc.task_size; s[2] = 0; s[3] = sell; s[4] = fbit(mid / (float)c.tick_size);
                for (int k = 5; k < 13; ++k) s[k] = fbit(0.0f);
            }
            const int nw = agent_words(tc);
            i32 v = 0;
            for (int k = 0; k < 13; ++k) if (l == k) v = s[k];
            if (l < nw) st[l] = v;
            if (obs) write_obs<false>(c, tc, wv, s, obs + (size_t)ag * c.obs_stride, false, ftime);
            st += nw;
        }
    }
}

template <int S>
__global__ __launch_bounds__(64) void k_env_reset(hftlob_env_cfg c, int n_env, const u32* __restrict__ keys,
                                                  const i32* __restrict__ init_states, i32* __restrict__ state,
                                                  float* __restrict__ obs) {
    one_wave();
    const int e = blockIdx.x;
    if (e >= n_env) return;
    Valid<S> VS, VT;
    VS.init(c.lob.n_orders);
    VT.init(c.lob.n_trades);
    Key k{keys[2 * e], keys[2 * e + 1]};
    env_reset_dev<S>(c, k, init_states, state + (size_t)e * c.rec_words,
                     obs ? obs + (size_t)e * c.n_agents * c.obs_stride : nullptr, VS, VT, c.ep_type == 1);
}

// ------------------------------------------------------------ agent logic
struct ActX {
    i32 bid_price, ask_price, bid_dist, ask_dist, bid_quant, ask_quant;
};

// write one 8-int message row into the LDS staging area (lane 0..7 each write a field)
DEV void put_row(i32* lds_rows, int row, i32 f0, i32 f1, i32 f2, i32 f3, i32 f4, i32 f5, i32 f6, i32 f7) {
    const int l = lane_id();
    i32 v = f0;
    v = l == 1 ? f1 : v; v = l == 2 ? f2 : v; v = l == 3 ? f3 : v;
    v = l == 4 ? f4 : v; v = l == 5 ? f5 : v; v = l == 6 ? f6 : v; v = l == 7 ? f7 : v;
    if (l < 8) lds_rows[row * 8 + l] = v;
}

// getCancelMsgs — JaxOrderBookArrays.py:827-853
template <int S>
DEV void cancel_rows(const Side<S>& s, int R, const Valid<S>& V, i32 agent, int size, i32 side, i32 t, i32 tns,
                     i32* lds_rows, int row0) {
    int n = 0;
    i32 tid[S], q[S], o[S];  // one LDS round trip; hit rows are read from registers
    const i32 (&p)[S] = s.pc;
    ldcol(s.t, R, FTID, tid);
    ldcol(s.t, R, FQ, q);
    ldcol(s.t, R, FOID, o);
#pragma unroll
    for (int r = 0; r < S; ++r) {
        lmask bm = V.m[r] & bal(tid[r] == agent);
        while (bm && n < size) {
            const int ln = (int)__builtin_ctzll(bm);
            bm &= bm - 1;
            put_row(lds_rows, row0 + n, 2, side, rdl(q[r], ln), rdl(p[r], ln), rdl(o[r], ln), agent, t, tns);
            ++n;
        }
    }
    for (; n < size; ++n) put_row(lds_rows, row0 + n, 2, side, 0, 0, 0, 0, t, tns);
}

// _filter_messages — mm_env.py:520-582 == exec_env.py:413-475, lane-parallel:
// lane i < n holds action row arow + i, lane 8 + j cancel row crow + j.
// Action i and cancel j match when their prices agree and the price is not 0;
// the k-th matched action pairs with the k-th matched cancel (in row order),
// rel[k] = (cv[k] >= av[k]) ? av[k] : 0 over the zero-padded k-th matched
// quantities, and every row subtracts rel[its rank] (unmatched rows rank after
// the matched ones).  Action rows left with quantity 0 become all-zero rows.
// `scratch`: 16 words of LDS.
template <int n>
DEV void filter_rows(i32* lds_rows, int arow, int crow, i32* scratch) {
    wave_sync();  // (one-wave workgroups: the rows written above are read back in order, no barrier)
    const int l = lane_id();
    const bool is_a = l < n, is_c = (l >= 8) & (l < 8 + n);
    const int row = is_a ? arow + l : (is_c ? crow + l - 8 : arow);
    const i32 p = lds_rows[row * 8 + 3], q = lds_rows[row * 8 + 2];
    lmask ma = 0, mc = 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        const i32 cpk = rdl(p, 8 + k), apk = rdl(p, k);
        ma |= bal(is_a & (p != 0) & (p == cpk));
        mc |= bal(is_c & (apk != 0) & (p == apk));
    }
    constexpr lmask amask = (1ull << n) - 1, cmask = amask << 8;
    const int na = __builtin_popcountll(ma), nc = __builtin_popcountll(mc);
    const lmask mine = is_a ? ma : mc, all = is_a ? amask : cmask;
    const bool matched = (mine >> l) & 1ull;
    const lmask below = matched ? mine : (~mine & all);
    const int cnt = (int)__builtin_amdgcn_mbcnt_hi((u32)(below >> 32), __builtin_amdgcn_mbcnt_lo((u32)below, 0u));
    const int rank = matched ? cnt : (is_a ? na : nc) + cnt;
    if (l < 16) scratch[l] = 0;  // av[k] = scratch[k], cv[k] = scratch[8 + k]
    wave_sync();
    if ((is_a | is_c) & matched) scratch[(is_c ? 8 : 0) + rank] = q;
    wave_sync();
    const i32 av = scratch[rank & 7], cv = scratch[8 + (rank & 7)];
    const i32 nq = wsub(q, cv >= av ? av : 0);
    if (is_a & (nq == 0)) {
        reinterpret_cast<int4*>(lds_rows + row * 8)[0] = make_int4(0, 0, 0, 0);
        reinterpret_cast<int4*>(lds_rows + row * 8)[1] = make_int4(0, 0, 0, 0);
    } else if (is_a | is_c) {
        lds_rows[row * 8 + 2] = nq;
    }
    wave_sync();
}

// MM _getActionMsgs_fixedQuant — mm_env.py:970-1118
// best ask / bid of the book with the agent's own orders masked out (get_best_bid_and_ask
// over the masked sides, mm_env.py:979-997), floored to the tick; an empty side falls back
// to the last recorded best quotes.  Returns empty_book.
template <int S>
DEV bool masked_best(const hftlob_env_cfg& c, Book<S>& B, i32 tid, i32 last_ba, i32 last_bb, i32& ba, i32& bb) {
    const i32 tick = c.tick_size;
    i32 mn = INT_MAX, mx = INT_MIN, at_[S], bt_[S];
    const i32 (&ap_)[S] = B.a.pc;
    const i32 (&bp_)[S] = B.b.pc;
    ldcol(B.a.t, B.c.nO, FTID, at_);
    ldcol(B.b.t, B.c.nO, FTID, bt_);
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const i32 pa = (B.vs.v[r] && at_[r] != tid) ? ap_[r] : -1;
        const i32 pb = (B.vs.v[r] && bt_[r] != tid) ? bp_[r] : -1;
        mn = imin_(mn, B.vs.v[r] ? (pa == -1 ? c.lob.maxint : pa) : INT_MAX);
        mx = imax_(mx, B.vs.v[r] ? pb : INT_MIN);
    }
    ba = wave_min(mn);
    bb = wave_max(mx);
    ba = ba == c.lob.maxint ? -1 : ba;
    const bool empty = (ba == -1) || (bb == -1);
    ba = wmul(tick_floordiv(c, ba), tick);
    bb = wmul(tick_floordiv(c, bb), tick);
    if (empty) { bb = last_bb; ba = last_ba; }
    return empty;
}
template <int S>
DEV void mm_fixed_quant(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, Book<S>& B, const i32* st, i32 tid,
                        i32 action, i32 wt0, i32 wt1, i32 last_ba, i32 last_bb, i32* lds_rows, int row, ActX& x) {
    if (tc.fixed_action_setting) action = tc.fixed_action;
    const i32 tick = c.tick_size;
    i32 ba, bb;
    const bool empty = masked_best(c, B, tid, last_ba, last_bb, ba, bb);
    const float hsp = fmaxf(i2f(wsub(ba, bb)) / 2.0f, (float)tick / 2.0f);
    const float hs = (tick_ffloordiv(c, hsp) + 1.0f) * (float)tick;
    float bo, ao;
    i32 bq, aq;
    if (!tc.sell_buy_all_option) {
        const int ai = action < 0 ? imax_(action + 10, 0) : (action > 9 ? 9 : action);  // jnp gather index
        // offsets tables {0,1,2,3,4,0,2,5,1,0} / {0,1,2,3,4,2,0,1,5,0}; quants 1.. ,0
        bo = (float)((0x0152043210ull >> (4 * ai)) & 0xF);
        ao = (float)((0x0510243210ull >> (4 * ai)) & 0xF);
        const i32 q1 = ai == 9 ? 0 : 1;
        bq = wmul(q1, tc.fixed_quant_value);
        aq = wmul(q1, tc.fixed_quant_value);
    } else {  // mm_env.py:1018-1023: 9-entry tables, entries 6 / 7 sell or buy the inventory back
        const int ai = action < 0 ? imax_(action + 9, 0) : (action > 8 ? 8 : action);
        const i32 bot[9] = {10, 2, 4, -1, 0, 2, -20, 0, 0}, aot[9] = {10, 2, 4, -1, 2, 0, 0, -20, 0};
        const i32 iq = ifloordiv(st[2], tc.fixed_quant_value);
        i32 b = bot[0], a = aot[0];  // table lookups as selects: a dynamically indexed local array lives in scratch
#pragma unroll
        for (int k = 1; k < 9; ++k) { b = ai == k ? bot[k] : b; a = ai == k ? aot[k] : a; }
        bo = i2f(b);
        ao = i2f(a);
        bq = wmul(ai < 6 ? 1 : (ai == 6 ? iq : 0), tc.fixed_quant_value);
        aq = wmul(ai < 6 ? 1 : (ai == 7 ? iq : 0), tc.fixed_quant_value);
    }
    if (empty) { bq = 0; aq = 0; }
    const float bpf = i2f(bb) - bo * hs;
    const float apf = i2f(ba) + ao * hs;
    const i32 bp = f2i(tick_ffloordiv(c, fmaxf(bpf, 0.0f)) * (float)tick);
    const i32 ap = f2i(tick_ffloordiv(c, fmaxf(i2f(wadd(bp, tick)), apf)) * (float)tick);
    i32 typ0 = 1, typ1 = 1, sd0 = 1, sd1 = -1, qq0 = bq, qq1 = aq, pp0 = bp, pp1 = ap;
    const i32 inv = st[2];
    const i32 lq0 = f2i(tc.auto_liquidate_alpha * i2f(imax_(wsub(0, inv), 0)));
    const i32 lq1 = f2i(tc.auto_liquidate_alpha * i2f(imax_(inv, 0)));
    const i32 lp0 = f2i(i2f(ba) + hs * 10.0f), lp1 = f2i(i2f(bb) - hs * 10.0f);
    const bool liq = (tc.tenth_action_market && action == 9) ||
                     (tc.auto_liquidate_threshold != 0 && iabs_(inv) > tc.auto_liquidate_threshold);
    if (liq) { typ0 = typ1 = 4; sd0 = -1; sd1 = 1; qq0 = lq0; qq1 = lq1; pp0 = lp0; pp1 = lp1; }
    const i32 ta = wadd(wt0, tc.time_delay_obs_act), tb = wadd(wt1, tc.time_delay_obs_act);
    put_row(lds_rows, row, typ0, sd0, qq0, pp0, c.placeholder_order_id, tid, ta, tb);
    put_row(lds_rows, row + 1, typ1, sd1, qq1, pp1, c.placeholder_order_id, tid, ta, tb);
    x.bid_price = bp; x.ask_price = ap; x.bid_dist = wsub(bb, bp); x.ask_dist = wsub(ap, ba);
    x.bid_quant = bq; x.ask_quant = aq;
}

// MM actions bobRL / bobStrategy / AvSt / spread_skew / simple (mm_env.py:1123-1809)
DEV i32 f2i_sat(float f) {  // XLA f32 -> s32 convert: saturating, NaN -> 0
    return f != f ? 0 : (f >= 2147483648.0f ? INT_MAX : (f <= -2147483648.0f ? INT_MIN : (i32)f));
}
template <int S>
DEV void mm_other_actions(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, Book<S>& B, const i32* st, i32 tid,
                          i32 action, i32 wt0, i32 wt1, i32 last_ba, i32 last_bb, i32 step, i32 init_t0, i32* lds_rows,
                          int row, ActX& x) {
    if (tc.fixed_action_setting) action = tc.fixed_action;
    const i32 tick = c.tick_size, inv = st[2], fq = tc.fixed_quant_value;
    const int kind = tc.action_space;
    // length of the indexed table: bobRL 2*v0+1, AvSt 8, simple 4 (3 without the do-nothing entry)
    const int na = kind == HFTLOB_MM_ACT_SIMPLE ? (tc.simple_nothing_action ? 4 : 3)
                                                 : (kind == HFTLOB_MM_ACT_AVST ? 8 : 2 * tc.bob_v0 + 1);
    // jnp gather index: negative wraps once, then clamps into range
    int ai = action < 0 ? action + na : action;
    ai = ai < 0 ? 0 : (ai >= na ? na - 1 : ai);
    i32 bp, ap, bq, aq, bdist = 0, adist = 0, bpost = 0, apost = 0;
    if (kind == HFTLOB_MM_ACT_BOB_RL || kind == HFTLOB_MM_ACT_BOB_STRATEGY || kind == HFTLOB_MM_ACT_AVST) {
        i32 ba, bb;
        const bool empty = masked_best(c, B, tid, last_ba, last_bb, ba, bb);
        if (kind == HFTLOB_MM_ACT_BOB_RL) {  // :1474-1561; tables bid v0 + (+k, -k, ...) / ask v0 - ...
            const i32 v0 = tc.bob_v0, d = (ai & 1) ? (ai + 1) / 2 : -(ai / 2);
            bq = wmul(wadd(v0, d), fq);
            aq = wmul(wsub(v0, d), fq);
            if (empty) { bq = 0; aq = 0; }
            bp = bb; ap = ba;
        } else if (kind == HFTLOB_MM_ACT_BOB_STRATEGY) {  // :1400-1472
            const float kappa = i2f(wadd(action, 1)) / i2f(wmul(tc.bob_v0, 5));
            const float pos = i2f(inv), v0 = (float)tc.bob_v0;
            bq = f2i_sat(rintf(v0 * fmaxf(1.0f - kappa * pos, 0.0f)));
            aq = f2i_sat(rintf(v0 * fmaxf(1.0f + kappa * pos, 0.0f)));
            if (empty) { bq = 0; aq = 0; }
            bp = bb; ap = ba;
        } else {  // AvSt :1248-1398
            const i32 mid = ifloordiv(wadd(ba, bb), 2);
            const float gam[8] = {0.1f, 0.2f, 0.5f, 1.0f, 2.0f, 5.0f, 10.0f, 20.0f};
            float gamma = gam[0], lt = tc.avst_log_term[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) if (ai == k) { gamma = gam[k]; lt = tc.avst_log_term[k]; }
            const i32 tl = c.ep_type == 1 ? wsub(c.episode_time, wsub(wt0, init_t0)) : wsub(c.episode_time, step);
            const float nt = i2f(tl) / i2f(c.episode_time);
            const float res = i2f(mid) - i2f(inv) * gamma * tc.avst_var * nt;
            float spread = gamma * tc.avst_var * nt + (2.0f / gamma) * lt;
            spread = fminf(fmaxf(spread, (float)tick), (float)c.lob.maxint);
            float bf = res - spread / 2.0f, af = res + spread / 2.0f;
            bf = fminf(fmaxf(bf, 0.0f), (float)c.lob.maxint);
            af = fminf(fmaxf(af, 0.0f), (float)c.lob.maxint);
            bp = f2i_sat(tick_ffloordiv(c, bf) * (float)tick);
            ap = f2i_sat(tick_ffloordiv(c, af) * (float)tick);
            const i32 q = tick_floordiv(c, mid), rm = wsub(mid, wmul(q, tick));
            bp = imin_(bp, wmul(wsub(q, rm == 0 ? 1 : 0), tick));  // round_down: strictly below mid
            ap = imax_(ap, wmul(wadd(q, 1), tick));                // round_up: strictly above mid
            bq = fq; aq = fq;
            bdist = wsub(bb, bp); adist = wsub(ap, ba); bpost = bp; apost = ap;
        }
    } else {
        const i32 ba = wmul(tick_floordiv(c, last_ba), tick), bb = wmul(tick_floordiv(c, last_bb), tick);
        if (kind == HFTLOB_MM_ACT_SPREAD_SKEW) {  // :1667-1808
            const float mid = i2f(wadd(ba, bb)) / 2.0f;
            const i32 cur = wsub(ba, bb);
            const i32 st_ = ifloordiv(action, 3), sk = wsub(action, wmul(st_, 3));
            const float mult = st_ == 0 ? 1.0f : tc.spread_multiplier;
            const float nsp = i2f(cur) * mult;
            const float skt = sk == 0 ? -tc.skew_multiplier : (sk == 1 ? 0.0f : tc.skew_multiplier);
            const float smid = mid + skt * (tc.multiplier_type ? nsp : (float)tick);
            const float hs = ffloordiv(nsp, 2.0f);
            bp = f2i_sat(tick_ffloordiv(c, smid - hs) * (float)tick);
            ap = f2i_sat(tick_ffloordiv(c, smid + hs) * (float)tick);
            bq = fq; aq = fq;
        } else {  // simple :1123-1246
            const float bo = ai == 1 ? -2000.0f : 0.0f, ao = ai == 2 ? -2000.0f : 0.0f;
            if (tc.sell_buy_all_option) {
                const i32 big = imax_(iabs_(inv), fq);
                const i32 bqa = inv > 0 ? fq : big, aqa = inv > 0 ? big : fq;
                bq = ai == 0 ? fq : (ai == 1 ? bqa : 0);
                aq = ai == 0 ? fq : (ai == 2 ? aqa : 0);
            } else {
                bq = wmul((ai == 0 || ai == 1) ? 1 : 0, fq);
                aq = wmul((ai == 0 || ai == 2) ? 1 : 0, fq);
            }
            // entry 3 (simple_nothing_action) is all zeros; with 3 entries `ai` clamps to 2
            const float to = (float)wmul(tc.n_ticks_offset, tick);
            const float bf = i2f(bb) - bo * to, af = i2f(ba) + ao * to;
            bp = f2i_sat(tick_ffloordiv(c, fmaxf(bf, 0.0f)) * (float)tick);
            ap = f2i_sat(tick_ffloordiv(c, af) * (float)tick);
        }
    }
    const i32 ta = wadd(wt0, tc.time_delay_obs_act), tb = wadd(wt1, tc.time_delay_obs_act);
    put_row(lds_rows, row, 1, 1, bq, bp, c.placeholder_order_id, tid, ta, tb);
    put_row(lds_rows, row + 1, 1, -1, aq, ap, c.placeholder_order_id, tid, ta, tb);
    x.bid_price = bpost; x.ask_price = apost; x.bid_dist = bdist; x.ask_dist = adist;
    x.bid_quant = bq; x.ask_quant = aq;
}

// MM _getActionMsgs_directional_trading — mm_env.py:1810-1865
DEV void mm_directional(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, i32 tid, i32 action, i32 wt0, i32 wt1,
                        i32 last_ba, i32 last_bb, i32* lds_rows, int row, ActX& x) {
    const i32 tick = c.tick_size;
    const i32 ba = wmul(tick_floordiv(c, last_ba), tick), bb = wmul(tick_floordiv(c, last_bb), tick);
    const int ai = action < 0 ? imax_(action + 3, 0) : (action > 2 ? 2 : action);
    const i32 bq = (ai == 1) * tc.fixed_quant_value, aq = (ai == 2) * tc.fixed_quant_value;
    const i32 ta = wadd(wt0, tc.time_delay_obs_act), tb = wadd(wt1, tc.time_delay_obs_act);
    put_row(lds_rows, row, 1, 1, bq, ba, c.placeholder_order_id, tid, ta, tb);
    put_row(lds_rows, row + 1, 1, -1, aq, bb, c.placeholder_order_id, tid, ta, tb);
    x.bid_price = x.ask_price = x.bid_dist = x.ask_dist = 0;
    x.bid_quant = bq; x.ask_quant = aq;
}

// EXE _getActionMsgs_fixedQuant_extended — exec_env.py:838-932
// + simplest_case (:935-999), fixed_quants_1msg (:732-836), twap (:1126-1227): rows = n_action_msgs
DEV void exe_fqc(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, const i32* st, i32 tid, i32 action, i32 wt0,
                 i32 wt1, i32 last_ba, i32 last_bb, i32 step, i32 max_steps, i32* lds_rows, int row) {
    const i32 tick = c.tick_size;
    const i32 ba = wmul(tick_floordiv(c, last_ba), tick), bb = wmul(tick_floordiv(c, last_bb), tick);
    const i32 sell = st[3];
    i32 pl[4];
    if (sell) {
        pl[0] = bb;
        pl[1] = f2i(ceilf(tick_ffloordiv(c, i2f(wadd(bb, ba)) / 2.0f)) * (float)tick);
        pl[2] = ba;
        pl[3] = wadd(ba, wmul(tick, tc.n_ticks_in_book));
    } else {
        pl[0] = ba;
        pl[1] = wmul(tick_floordiv(c, ifloordiv(wadd(bb, ba), 2)), tick);
        pl[2] = bb;
        pl[3] = wsub(bb, wmul(tick, tc.n_ticks_in_book));
    }
    const i32 side = wsub(1, wmul(sell, 2));
    const i32 ta = wadd(wt0, tc.time_delay_obs_act), tb = wadd(wt1, tc.time_delay_obs_act);
    const i32 fq = tc.fixed_quant_value, left = wsub(st[1], st[2]);
    i32 q[4] = {0, 0, 0, 0};
    if (tc.action_space == HFTLOB_EXE_ACT_FIXED_QUANTS_COMPLEX) {
        const int ai = action < 0 ? imax_(action + 13, 0) : (action > 12 ? 12 : action);
        // quant table rows: action 0 -> none; 1..12 -> level (ai-1)%4 with multiple {1,2,5}[(ai-1)/4]
        if (ai > 0) {
            const int lvl = (ai - 1) & 3, mul = (ai - 1) >> 2;
            const i32 v = wmul(mul == 0 ? 1 : (mul == 1 ? 2 : 5), fq);
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = k == lvl ? v : 0;  // (selects: no dynamically indexed array)
        }
        const i32 tot = wadd(wadd(q[0], q[1]), wadd(q[2], q[3]));
        if (!(tot <= left)) { q[0] = f2i(floorf(i2f(left))); q[1] = q[2] = q[3] = 0; }
        for (int k = 0; k < 4; ++k) put_row(lds_rows, row + k, 1, side, q[k], pl[k], c.placeholder_order_id, tid, ta, tb);
        return;
    }
    if (tc.action_space == HFTLOB_EXE_ACT_FIXED_QUANTS_1MSG) {  // one row at [0, FT, M, NT, PP][a]
        const int ai = action < 0 ? imax_(action + 5, 0) : (action > 4 ? 4 : action);
        i32 p = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) p = ai == k + 1 ? pl[k] : p;
        i32 qq = ai == 0 ? 0 : fq;
        qq = qq <= left ? qq : 0;
        put_row(lds_rows, row, 1, side, qq, p, c.placeholder_order_id, tid, ta, tb);
        return;
    }
    // two rows at (FT, NT)
    const i32 ft = sell ? bb : ba, nt = sell ? ba : bb;
    if (tc.action_space == HFTLOB_EXE_ACT_SIMPLEST_CASE) {
        const int ai = action < 0 ? imax_(action + 3, 0) : (action > 2 ? 2 : action);
        q[0] = ai == 1 ? fq : 0;
        q[1] = ai == 2 ? fq : 0;
        if (!(wadd(q[0], q[1]) <= left)) { q[0] = f2i(floorf(i2f(wmul(fq, left)))); q[1] = 0; }
    } else {  // twap: ceil(max(task - executed, 0) / steps_left) at FT (action 0) or NT (action 1)
        const int ai = action < 0 ? imax_(action + 2, 0) : (action > 1 ? 1 : action);
        const i32 steps_left = wsub(wsub(max_steps, step), 1);
        const i32 qts = f2i_sat(ceilf(i2f(imax_(left, 0)) / i2f(steps_left)));
        q[0] = ai == 0 ? qts : 0;
        q[1] = ai == 1 ? qts : 0;
    }
    put_row(lds_rows, row, 1, side, q[0], ft, c.placeholder_order_id, tid, ta, tb);
    put_row(lds_rows, row + 1, 1, side, q[1], nt, c.placeholder_order_id, tid, ta, tb);
}

// EXE _getActionMsgs_fixedPrice — exec_env.py:1001-1123.  act[0..w) is the
// MultiDiscrete action, w = n_actions (1..4): the quantity at each of the first w
// price levels of (FT, M, NT, PP) / (FT, NT, PP) / (FT, NT) / (FT).  Quantities are
// rescaled in f32 to the quantity left when they sum past it; the reference prices
// are the f32 means of the last 10 best quotes of the previous step, floored to the tick.
DEV void exe_fixed_prices(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, const i32* rec, const i32* st,
                          i32 tid, const i32 (&act)[4], i32 wt0, i32 wt1, i32* lds_rows, int row) {
    const i32 tick = c.tick_size, w = tc.n_actions, left = wsub(st[1], st[2]), sell = st[3];
    i32 sum = 0;
    for (int j = 0; j < w; ++j) sum = wadd(sum, act[j]);
    i32 q[4];
    const bool rescale = sum > left;
    for (int j = 0; j < 4; ++j) q[j] = rescale ? f2i_sat(i2f(act[j]) / i2f(sum) * i2f(left)) : act[j];
    // best_asks[-10:].mean(axis=0)[0]: f32 sum in row order, / n  (:1089-1090)
    const int M = c.n_msgs, m0 = M > 10 ? M - 10 : 0;
    float sa = 0.0f, sb = 0.0f;
    for (int m = m0; m < M; ++m) {
        sa += i2f(rec[c.off_best_asks + m * 2]);
        sb += i2f(rec[c.off_best_bids + m * 2]);
    }
    const float n = (float)(M - m0), ft = (float)tick;
    const i32 ba = f2i_sat(ffloordiv(sa / n, ft) * ft), bb = f2i_sat(ffloordiv(sb / n, ft) * ft);
    i32 lv[4];  // FT, M, NT, PP
    if (sell) {
        lv[0] = wmul(tick_floordiv(c, bb), tick);
        lv[1] = f2i_sat(ceilf(ffloordiv(i2f(wadd(bb, ba)) / 2.0f, ft)) * ft);
        lv[2] = ba;
        lv[3] = wadd(ba, wmul(tick, tc.n_ticks_in_book));
    } else {
        lv[0] = wmul(tick_floordiv(c, ba), tick);
        lv[1] = wmul(tick_floordiv(c, ifloordiv(wadd(bb, ba), 2)), tick);
        lv[2] = bb;
        lv[3] = wsub(bb, wmul(tick, tc.n_ticks_in_book));
    }
    i32 p[4];
    if (w == 4) { p[0] = lv[0]; p[1] = lv[1]; p[2] = lv[2]; p[3] = lv[3]; }
    else { p[0] = lv[0]; p[1] = lv[2]; p[2] = lv[3]; p[3] = 0; }
    if (w == 4 && lv[1] == lv[2]) {  // mid == near touch: one order at the near touch
        q[2] = wadd(q[2], q[1]);
        q[1] = 0;
        p[1] = -1;
    }
    const i32 side = wsub(1, wmul(sell, 2));
    const i32 ta = wadd(wt0, tc.time_delay_obs_act), tb = wadd(wt1, tc.time_delay_obs_act);
    for (int j = 0; j < w; ++j) put_row(lds_rows, row + j, 1, side, q[j], p[j], c.placeholder_order_id, tid, ta, tb);
}

// --------------------------------------------------------------- rewards
// Per-row trade views with an optional override row (the fictional unwind
// trade that add_trade — JaxOrderBookArrays.py:885-889 — places at the first
// row holding any -1; the override is per agent and never stored).
template <int S>
struct TradeView {
    i32 P[S], Q[S], S4[S], PT[S], AT[S];
    bool valid[S];  // trades[:,0] >= 0 ("executed")
};
template <int S>
DEV void trade_view(const Book<S>& B, TradeView<S>& V, bool use_ovr, int ovr_idx, const i32 (&ovr)[8]) {
    const int l = lane_id();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const bool o = use_ovr && (r * 64 + l == ovr_idx);
        const i32 p = o ? ovr[0] : B.tr.get(0, r), q = o ? ovr[1] : B.tr.get(1, r);
        const i32 s4 = o ? ovr[4] : B.tr.get(4, r), pt = o ? ovr[6] : B.tr.get(6, r), at = o ? ovr[7] : B.tr.get(7, r);
        const bool v = B.vt.v[r] && p >= 0;
        V.valid[r] = v;
        V.P[r] = v ? p : 0; V.Q[r] = v ? q : 0; V.S4[r] = v ? s4 : 0; V.PT[r] = v ? pt : 0; V.AT[r] = v ? at : 0;
    }
}
template <int S> DEV int first_any_neg1_trade(const Book<S>& B) {
    bool pr[S];
#pragma unroll
    for (int r = 0; r < S; ++r) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < 8; ++k) any |= B.tr.get(k, r) == -1;
        pr[r] = B.vt.v[r] && any;
    }
    return first_true(pr, B.c.nT - 1);
}

struct StepCtx {  // wave-uniform per-step quantities shared by the rewards
    float avg_mid, last_mid, wmid;
    i32 last_ba, last_bb, old_last_ba, old_last_bb;  // new / old best quotes [-1]
    i32 init0, step;
    bool ep_done;
};

struct MMRew {
    float reward, reward_pv, reward_spooner, end_of_ep_pv, reward_spooner_damped, reward_spooner_asym_damped,
        reward_spooner_asym_damped2, reward_delta_pv, market_share, delta_mid, buyPnL, sellPnL, invPnL, PnL, cash,
        inventoryValue;
    i32 end_inventory, forced_unwind;
};

// MM get_reward — mm_env.py:2214-2673
template <int S>
DEV void mm_reward(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, const Book<S>& B, const StepCtx& X,
                   const i32* st, i32 tid, bool excl_any, const TradeView<S>& TV, MMRew& R, bool full = true) {
    const int nT = c.lob.n_trades;
    const float tick = (float)c.tick_size;
    TradeView<S> V = TV;  // the step's trades (the unwind below overrides one row of this agent's copy)
    const i32 inv = st[2];
    const i32 M = c.n_msgs;
    // the forced unwind exists only on an episode's last step: the pre-unwind inventory and the
    // second trade view are skipped on every other step (forced_unwind = inv_b * ep_done = 0)
    R.forced_unwind = 0;
    if (X.ep_done) {
        i32 bqs = 0, sqs = 0;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const bool mine = (tid == V.PT[r]) || (tid == V.AT[r]);
            const i32 aQ = mine ? V.Q[r] : 0, apt = mine ? V.PT[r] : 0, aat = mine ? V.AT[r] : 0;
            const bool buy = (aQ >= 0 && tid == apt) || (aQ < 0 && tid == aat);
            const bool sel = (aQ < 0 && tid == apt) || (aQ >= 0 && tid == aat);
            bqs = wadd(bqs, buy ? iabs_(aQ) : 0);
            sqs = wadd(sqs, sel ? iabs_(aQ) : 0);
        }
        bqs = wave_sum(bqs);
        sqs = wave_sum(sqs);
        const i32 inv_b = wsub(wadd(inv, bqs), sqs);
        i32 pen = wmul(tc.unwind_price_penalty, c.tick_size);
        pen = inv_b > 0 ? pen : wsub(0, pen);
        i32 unwind_px;
        if (tc.unwind_price == HFTLOB_PRICE_FAR_TOUCH) unwind_px = wsub(sel(inv_b > 0, X.last_bb, X.last_ba), pen);
        else unwind_px = f2i(self(tc.unwind_price == HFTLOB_PRICE_MID_AVG, X.avg_mid, X.last_mid) - i2f(pen));
        if (iabs_(inv_b) > 0) {
            const i32 ovr[8] = {unwind_px, wmul(isign(inv_b), iabs_(inv_b)), c.artificial_order_id,
                                c.placeholder_order_id, 0, 0, c.artificial_trader_id, tid};
            trade_view(B, V, true, first_any_neg1_trade(B), ovr);
        }
        R.forced_unwind = inv_b;
    }
    // post-unwind stats
    const int ri = tc.reference_price;
    const bool ref_int = ri == HFTLOB_PRICE_FAR_TOUCH || ri == HFTLOB_PRICE_NEAR_TOUCH;
    i32 bq = 0, sq = 0, oq = 0;
    i32 bP[S], bQ[S], sP[S], sQ[S];
    float income, outgoing, rebate_value;
    lmask anym = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) anym |= bal((tid == V.PT[r]) || (tid == V.AT[r]));
    const bool quiet = anym == 0ull;
    if (quiet) {
        // no row is the agent's (no fill this step: 98 % of the metric's steps): every buy / sell
        // stat is 0 and every float row term below is one and the same signed zero, summed by
        // zsum exactly as rows_fsum would
#pragma unroll
        for (int r = 0; r < S; ++r) {
            oq = wadd(oq, iabs_(V.Q[r]));
            bP[r] = bQ[r] = sP[r] = sQ[r] = 0;
        }
        oq = wave_sum(oq);
        // (0 / tick * 0 = +0: tick >= 1)
        income = outgoing = zsum(0.0f, nT);
        rebate_value = zsum(0.0f, nT) + zsum(0.0f, nT);
    } else {
        float inc[S], out[S], rb[S], rsl[S];
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const bool mine = (tid == V.PT[r]) || (tid == V.AT[r]);
            const i32 aP = mine ? V.P[r] : 0, aQ = mine ? V.Q[r] : 0, apt = mine ? V.PT[r] : 0, aat = mine ? V.AT[r] : 0;
            oq = wadd(oq, mine ? 0 : iabs_(V.Q[r]));
            const bool buy = (aQ >= 0 && tid == apt) || (aQ < 0 && tid == aat);
            const bool sel = (aQ < 0 && tid == apt) || (aQ >= 0 && tid == aat);
            const bool pbuy = (aQ >= 0 && tid == apt), psel = (aQ < 0 && tid == apt);
            bP[r] = buy ? aP : 0; bQ[r] = buy ? aQ : 0; sP[r] = sel ? aP : 0; sQ[r] = sel ? aQ : 0;
            const i32 pbP = pbuy ? aP : 0, pbQ = pbuy ? aQ : 0, psP = psel ? aP : 0, psQ = psel ? aQ : 0;
            bq = wadd(bq, iabs_(bQ[r]));
            sq = wadd(sq, iabs_(sQ[r]));
            inc[r] = i2f(sP[r]) / tick * i2f(iabs_(sQ[r]));
            out[r] = i2f(bP[r]) / tick * i2f(iabs_(bQ[r]));
            rb[r] = i2f(pbP) / tick * i2f(iabs_(pbQ));
            rsl[r] = i2f(psP) / tick * i2f(iabs_(psQ));
        }
        bq = wave_sum(bq); sq = wave_sum(sq); oq = wave_sum(oq);
        income = rows_fsum(inc, nT);
        outgoing = rows_fsum(out, nT);
        rebate_value = rows_fsum(rb, nT) + rows_fsum(rsl, nT);
    }
    const i32 new_inv = wsub(wadd(inv, bq), sq);
    const float rebate_income = rebate_value * tc.rebate_factor;
    const float PnL = income - outgoing + rebate_income;
    const float cash = bitf(st[4]) + PnL;
    // the reward values: only when the step's outputs are emitted (the state needs PnL, cash and the
    // inventory).  One assignment block for both cases below: with an early return the compiler
    // merged the two paths' stores to different fields of R into stores through a selected address,
    // which puts R in scratch memory
    float reward = 0.0f, r_pv = 0.0f, r_sp = 0.0f, r_spd = 0.0f, r_spad = 0.0f, r_spad2 = 0.0f, d_nw = 0.0f,
          market_share = 0.0f, buyPnL = 0.0f, sellPnL = 0.0f, invPnL = 0.0f, inv_value = 0.0f;
    if (full) {
        float ref_buy, ref_sell, ref;
        i32 rbi = 0, rsi = 0, refi = 0;
        if (ri == HFTLOB_PRICE_MID_AVG) { ref_buy = ref_sell = ref = X.avg_mid; }
        else if (ref_int) {
            const bool far = ri == HFTLOB_PRICE_FAR_TOUCH;
            rbi = sel(far, X.last_ba, X.last_bb);
            rsi = sel(far, X.last_bb, X.last_ba);
            refi = new_inv > 0 ? rbi : rsi;
            ref_buy = i2f(rbi); ref_sell = i2f(rsi); ref = i2f(refi);
        } else { ref_buy = ref_sell = ref = X.last_mid; }
        const i32 traded = wadd(bq, sq);
        const float mid_end = X.last_mid;
        float old_ref;
        if (ri == HFTLOB_PRICE_FAR_TOUCH) old_ref = i2f(sel(inv > 0, X.old_last_ba, X.old_last_bb));
        else if (ri == HFTLOB_PRICE_NEAR_TOUCH) old_ref = i2f(sel(inv > 0, X.old_last_bb, X.old_last_ba));
        else old_ref = X.wmid;
        DivBatch D{lane_id()};
        D.add(0, ref_int ? i2f(wmul(new_inv, refi)) : i2f(new_inv) * ref, tick);  // inventoryValue
        D.add(1, i2f(traded), i2f(wadd(traded, oq)));                              // market_share
        D.add(2, i2f(inv) * (mid_end - X.wmid), tick);                             // InventoryPnL
        D.add(3, ref, tick);                                                       // portfolio value's ref / tick
        D.add(4, old_ref, tick);                                                   // the old net worth's
        D.run();
        inv_value = D.get(0);
        const float net_worth = cash + inv_value;
        market_share = D.get(1);
        invPnL = D.get(2);
        if (quiet) {  // (the rows' one signed zero: sign of the reference price term)
            // (x / tick * +0 is the zero of x's sign: x finite, tick >= 1, |x| >= 1 or x = +-0)
            const float zb = copysignf(0.0f, ref_int ? i2f(wsub(rbi, 0)) : ref_buy - i2f(0));
            const float zs = copysignf(0.0f, ref_int ? i2f(wsub(0, rsi)) : i2f(0) - ref_sell);
            buyPnL = zsum(zb, nT);
            sellPnL = zsum(zs, nT);
        } else {
            float bpl[S], spl[S];
    #pragma unroll
            for (int r = 0; r < S; ++r) {
                if (ref_int) {
                    bpl[r] = i2f(wsub(rbi, bP[r])) / tick * i2f(iabs_(bQ[r]));
                    spl[r] = i2f(wsub(sP[r], rsi)) / tick * i2f(iabs_(sQ[r]));
                } else {
                    bpl[r] = (ref_buy - i2f(bP[r])) / tick * i2f(iabs_(bQ[r]));
                    spl[r] = (i2f(sP[r]) - ref_sell) / tick * i2f(iabs_(sQ[r]));
                }
            }
            buyPnL = rows_fsum(bpl, nT);
            sellPnL = rows_fsum(spl, nT);
        }
        const float eta = tc.inventoryPnL_eta, gam = tc.inventoryPnL_gamma;
        r_sp = buyPnL + sellPnL + rebate_income + invPnL;
        r_spd = buyPnL + sellPnL + rebate_income + invPnL - eta * invPnL;
        r_spad = buyPnL + sellPnL + rebate_income + invPnL - fmaxf(0.0f, eta * invPnL);
        r_spad2 = buyPnL + sellPnL + rebate_income + gam * (invPnL - fmaxf(0.0f, eta * invPnL));
        const float r_sps = buyPnL + sellPnL + rebate_income + eta * (invPnL - tc.one_minus_eta * fmaxf(0.0f, invPnL));
        float r_complex = 0.0f;
        if (tc.reward_function == HFTLOB_MM_REW_COMPLEX) {
            float abp[S], asp[S];
    #pragma unroll
            for (int r = 0; r < S; ++r) {
                abp[r] = i2f(bP[r]) / i2f(bq) * i2f(iabs_(bQ[r]));
                asp[r] = i2f(sP[r]) / i2f(sq) * i2f(iabs_(sQ[r]));
            }
            const float avg_buy = bq > 0 ? rows_fsum(abp, nT) : 0.0f;
            const float avg_sell = sq > 0 ? rows_fsum(asp, nT) : 0.0f;
            const i32 inv_change = wsub(bq, sq);
            const float real_pnl = i2f(imin_(bq, sq)) * (avg_sell - avg_buy);
            const float unreal = inv_change > 0 ? i2f(inv_change) * (X.avg_mid - avg_buy)
                                                : i2f(iabs_(inv_change)) * (avg_sell - X.avg_mid);
            r_complex = real_pnl + tc.unrealizedPnL_lambda * unreal + eta * fminf(invPnL, invPnL * eta);
        }
        r_pv = i2f(new_inv) * D.get(3) + cash;
        const float old_nw = D.get(4) * i2f(inv) + bitf(st[4]);
        d_nw = net_worth - old_nw;
        switch (tc.reward_function) {
            case HFTLOB_MM_REW_PORTFOLIO_VALUE: reward = r_pv; break;
            case HFTLOB_MM_REW_BUY_SELL_PNL: reward = buyPnL + sellPnL; break;
            case HFTLOB_MM_REW_COMPLEX: reward = r_complex; break;
            case HFTLOB_MM_REW_ZERO_INV: reward = i2f(wsub(0, iabs_(new_inv))); break;
            case HFTLOB_MM_REW_SPOONER: reward = r_sp; break;
            case HFTLOB_MM_REW_SPOONER_DAMPED: reward = r_spd; break;
            case HFTLOB_MM_REW_SPOONER_ASYM_DAMPED: reward = r_spad; break;
            case HFTLOB_MM_REW_SPOONER_SCALED: reward = r_sps; break;
            case HFTLOB_MM_REW_DELTA_PORTFOLIO_VALUE: reward = d_nw; break;
            default: reward = r_spad2; break;
        }
        float inv_pen = 0.0f;
        if (tc.inv_penalty == HFTLOB_INVPEN_LINEAR) inv_pen = i2f(wsub(0, iabs_(new_inv)));
        else if (tc.inv_penalty == HFTLOB_INVPEN_QUADRATIC)
            inv_pen = i2f(wmul(-1, wmul(new_inv, new_inv))) / tc.inv_penalty_quadratic_factor;
        else if (tc.inv_penalty == HFTLOB_INVPEN_THRESHOLD)
            inv_pen = i2f(iabs_(new_inv)) > tc.inv_penalty_threshold
                          ? -1.0f * (i2f(wmul(new_inv, new_inv)) / tc.inv_penalty_quadratic_factor) : 0.0f;
        else if (tc.inv_penalty == HFTLOB_INVPEN_EXP4)  // mm_env.py:2528-2529: -exp(inv * 4), int32 product
            inv_pen = -1.0f * expf(i2f(wmul(new_inv, 4)));
        reward = reward + tc.inv_penalty_lambda * inv_pen;
        if (tc.clip_reward) reward = fminf(fmaxf(reward, -10000.0f), 10000.0f);
        if (tc.volume_traded_bonus == 1) reward = reward + fabsf(reward) * market_share;
        if (tc.exclude_extreme_spreads && excl_any) reward = 0.0f;
    }
    R.reward = reward; R.reward_pv = r_pv; R.reward_spooner = r_sp; R.end_of_ep_pv = r_pv * (float)X.ep_done;
    R.reward_spooner_damped = r_spd; R.reward_spooner_asym_damped = r_spad; R.reward_spooner_asym_damped2 = r_spad2;
    R.reward_delta_pv = d_nw; R.market_share = market_share; R.delta_mid = X.last_mid - X.wmid; R.buyPnL = buyPnL;
    R.sellPnL = sellPnL; R.invPnL = invPnL; R.PnL = PnL; R.cash = cash; R.inventoryValue = inv_value;
    R.end_inventory = new_inv;
    (void)M;
}

struct EXRew {
    float reward, reward_info, p_vwap, vwap_rm, price_adv_rm, slippage_rm, price_drift_rm, advantage, drift, slippage,
        trade_duration;
    i32 agentQuant, qp_agent, doom_quant, quant_left;
};

// EXE get_reward — exec_env.py:1511-1762
template <int S>
DEV void exe_reward(const hftlob_env_cfg& c, const hftlob_agent_type_cfg& tc, const Book<S>& B, const StepCtx& X,
                    const i32* st, i32 tid, const TradeView<S>& TV, EXRew& R, bool full = true) {
    const int nT = c.lob.n_trades;
    const i32 tick = c.tick_size;
    TradeView<S> V = TV;  // the step's trades (the doom trade below overrides one row of this agent's copy)
    const i32 task = st[1], qe = st[2], sell = st[3];
    const float init_price = bitf(st[0]);
    // the fictional doom trade exists only on an episode's last step: the pre-unwind quantity and
    // the second trade view are skipped on every other step (doom_quant = ep_done * quant_left = 0)
    R.doom_quant = 0;
    if (X.ep_done) {
        i32 qsum = 0;
#pragma unroll
        for (int r = 0; r < S; ++r) qsum = wadd(qsum, (tid == V.PT[r] || tid == V.AT[r]) ? V.Q[r] : 0);
        const i32 qets = iabs_(wave_sum(qsum));
        const i32 quant_left = wsub(task, wadd(qe, qets));
        const i32 pen = wmul(tc.doom_price_penalty, tick);
        const i32 side_sign = wsub(wmul(sell, 2), 1);
        i32 refp;
        const float penf = tc.doom_penalty_is_float ? tc.doom_penalty_f32 : i2f(pen);
        if (tc.reference_price == HFTLOB_PRICE_FAR_TOUCH && !tc.doom_penalty_is_float)
            refp = sell ? wmul(tick_floordiv(c, wsub(X.last_bb, pen)), tick)
                        : wmul(tick_floordiv(c, wadd(X.last_ba, pen)), tick);
        else if (tc.reference_price == HFTLOB_PRICE_FAR_TOUCH)  // int32 price - Python float: f32
            refp = sell ? f2i(tick_ffloordiv(c, i2f(X.last_bb) - penf) * (float)tick)
                        : f2i(tick_ffloordiv(c, i2f(X.last_ba) + penf) * (float)tick);
        else
            refp = sell ? f2i(tick_ffloordiv(c, X.avg_mid - penf) * (float)tick)
                        : f2i(tick_ffloordiv(c, X.avg_mid + penf) * (float)tick);
        if (quant_left > 0) {
            const i32 ovr[8] = {refp, wmul(side_sign, iabs_(quant_left)), c.artificial_order_id,
                                c.placeholder_order_id, 0, 0, c.artificial_trader_id, tid};
            trade_view(B, V, true, first_any_neg1_trade(B), ovr);
        }
        R.doom_quant = quant_left;
    }
    i32 aq = 0, oq = 0, qp = 0;
    lmask anym = 0;
#pragma unroll
    for (int r = 0; r < S; ++r) anym |= bal(V.valid[r] && (tid == V.PT[r] || tid == V.AT[r]));
    float dur_sum;
    if (anym == 0ull) {  // no fill of the agent this step: aq = qp = 0, every duration term the same signed zero
#pragma unroll
        for (int r = 0; r < S; ++r) oq = wadd(oq, iabs_(V.Q[r]));
        oq = wave_sum(oq);
        dur_sum = zsum(i2f(0) / i2f(task) * i2f(wsub(0, X.init0)), nT);
    } else {
        float dur[S];
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const bool mine = V.valid[r] && (tid == V.PT[r] || tid == V.AT[r]);
            aq = wadd(aq, mine ? iabs_(V.Q[r]) : 0);
            oq = wadd(oq, mine ? 0 : iabs_(V.Q[r]));
            qp = wadd(qp, mine ? wmul(tick_floordiv(c, V.P[r]), iabs_(V.Q[r])) : 0);
            dur[r] = mine ? i2f(iabs_(V.Q[r])) / i2f(task) * i2f(wsub(V.S4[r], X.init0))
                          : i2f(0) / i2f(task) * i2f(wsub(0, X.init0));
        }
        aq = wave_sum(aq); oq = wave_sum(oq); qp = wave_sum(qp);
        dur_sum = rows_fsum(dur, nT);
    }
    float pv;
    if (oq == 0) pv = tick_ffloordiv(c, X.avg_mid);
    else {
        float vw[S];
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const bool other = V.valid[r] && !(tid == V.PT[r] || tid == V.AT[r]);
            const i32 P = other ? V.P[r] : 0, Q = other ? V.Q[r] : 0;
            vw[r] = i2f(tick_floordiv(c, P)) * (i2f(iabs_(Q)) / i2f(oq));
        }
        pv = rows_fsum(vw, nT);
    }
    const i32 dirs = isign(wsub(wmul(sell, 2), 1));
    const float adv = i2f(dirs) * (i2f(qp) - pv * i2f(aq));
    const float drift = i2f(wmul(dirs, aq)) * (pv - tick_ffloordiv(c, init_price));
    const float slip = adv + drift;
    const float scf = i2f(X.step), sc1 = i2f(wadd(X.step, 1));
    DivBatch D{lane_id()};  // the per-agent averages, then the rolling means (exec_env.py:1760-1762)
    D.add(0, adv, i2f(aq) + 1e-9f);
    D.add(1, drift, i2f(aq) + 1e-9f);
    D.add(2, bitf(st[11]) * scf + pv, sc1);
    D.add(3, bitf(st[8]) * scf + slip, sc1);
    D.run();
    const float padv = D.get(0), pdrift = D.get(1);
    R.vwap_rm = D.get(2);
    R.slippage_rm = D.get(3);
    DivBatch D2{lane_id()};
    D2.add(0, bitf(st[9]) * scf + padv, sc1);
    D2.add(1, bitf(st[10]) * scf + pdrift, sc1);
    D2.run();
    R.price_adv_rm = D2.get(0);
    R.price_drift_rm = D2.get(1);
    float reward = adv + tc.reward_lambda * drift;
    R.trade_duration = bitf(st[12]) + dur_sum;
    R.quant_left = wsub(wsub(task, qe), aq);
    R.reward_info = reward;
    if (tc.reward_function == HFTLOB_EXE_REW_FINISH_FAST) reward = i2f(wsub(0, iabs_(R.quant_left)));
    if (full && tc.reward_function == HFTLOB_EXE_REW_SIMPLEST_CASE) {  // :1723-1731: sum (p - init_price) |q|, sign by task
        float ps[S];
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const bool mine = V.valid[r] && (tid == V.PT[r] || tid == V.AT[r]);
            const float slip = i2f(mine ? V.P[r] : 0) - init_price;
            ps[r] = (sell ? slip : -slip) * i2f(mine ? iabs_(V.Q[r]) : 0);
        }
        reward = rows_fsum(ps, nT);
    }
    R.reward = reward; R.p_vwap = pv; R.advantage = adv; R.drift = drift; R.slippage = slip;
    R.agentQuant = aq; R.qp_agent = qp;
}

// ------------------------------------------------------- step PRNG (VALU)
// Every key of one step, derived lane-parallel: lanes compute different
// threefry blocks at once, in VALU (the scalar unit is the shared resource of
// a CU; one threefry2x32-20 is ~100 instructions).  Derivation, as the
// scalar form in hftlob_sample_actions / k_env_step used it:
//   key        = keys[e], or split(master, n_env + 1)[e + 1] (rollout mode)
//   k1, key_reset = split(key)                           (marl_env.py:787)
//   sub        = split(split(k1)[1])[1]; bits[l] = random_bits(sub, A)[l]
//                (jax.random.permutation of the action rows, marl_env.py:293-295)
//   actions    = randint(split(split(key, n_types)[t], n_agents_t)[i], 0, n_actions_t)
//                (Speed_test.py:166-177), agent ag's in lane 32 + ag
struct StepKeys {
    Key key, k1, key_reset;
    Key next_master;   // rollout mode: split(master, n_env + 1)[0], the key the next step splits
    u32 shuffle_bits;  // lane l < A: random word of action row l
    i32 acts;          // lane 32 + ag: sampled action (rollout mode)
};
// agent lane 32 + ag -> (type, index within type)
// (per-lane type fields: each type's field is a uniform (scalar) load and the lane selects by its
// t; indexing c.types[t] with a lane-varying t would be a vector load from the kernel arguments,
// waited on at once, per use)
// (sel: a select of the loaded VALUES; as a plain ?: the compiler selects the field's address
// per lane and issues the vector load anyway)
DEV i32 type_n_agents(const hftlob_env_cfg& c, int t) {
    i32 v = c.types[0].n_agents;
#pragma unroll
    for (int k = 1; k < HFTLOB_MAX_TYPES; ++k) v = sel(t == k, c.types[k].n_agents, v);
    return v;
}
DEV i32 type_action_hi(const hftlob_env_cfg& c, int t, bool md) {
    i32 v = md ? action_hi(c.types[0]) : c.types[0].n_actions;
#pragma unroll
    for (int k = 1; k < HFTLOB_MAX_TYPES; ++k) v = sel(t == k, md ? action_hi(c.types[k]) : c.types[k].n_actions, v);
    return v;
}
DEV void agent_of_lane(const hftlob_env_cfg& c, int ag, int& t, int& i) {
    t = 0;
    i = ag;
#pragma unroll
    for (int k = 0; k < HFTLOB_MAX_TYPES - 1; ++k) {
        const i32 nk = c.types[k].n_agents;  // (t == k while every earlier test held)
        if ((k < c.n_types - 1) & (t == k) & (i >= nk)) { i -= nk; ++t; }
    }
}
DEV Key lane_key(Key v) { return Key{(u32)rdl((i32)v.a, 0), (u32)rdl((i32)v.b, 0)}; }
DEV Key from_lane(Key v, int src) {  // per-lane gather v[src]
    return Key{(u32)__builtin_amdgcn_ds_bpermute(src << 2, (i32)v.a), (u32)__builtin_amdgcn_ds_bpermute(src << 2, (i32)v.b)};
}
template <bool MD>  // MD: the config may hold MultiDiscrete (fixed_prices) agent types
DEV StepKeys step_keys(const hftlob_env_cfg& c, int n_env, int e, const u32* keys, bool sampled, const Key& master) {
    const bool part = c.prng_partitionable;
    const int l = lane_id(), nTy = c.n_types, A = c.n_action_msgs;
    Key key;
    Key nm{0u, 0u};
    if (sampled) {  // lane 0: this env's key; lane 1: the carried master key
        const Key v = split_key(master, n_env + 1, l == 0 ? e + 1 : 0, part);
        key = lane_key(v);
        nm = Key{(u32)rdl((i32)v.a, 1), (u32)rdl((i32)v.b, 1)};
    } else {
        key = Key{keys[2 * e], keys[2 * e + 1]};
    }
    // partitionable keys and <= 16 agents: agent ag's randint takes two lanes, 32 + ag (the high
    // word's key, split(k_ag)[0]) and 48 + ag (the low word's, split(k_ag)[1]), so levels 3 and 4
    // below are one threefry per lane each (5 per step instead of 8; the chain depth is the same)
    const bool two = part && c.n_agents <= 16 && A <= 32;
    const bool hi_lane = two && l >= 48;
    const int ag = l - (hi_lane ? 48 : 32);
    int t = 0, i = 0;
    agent_of_lane(c, ag < 0 ? 0 : ag, t, i);
    const bool agent_lane = (ag >= 0) & (ag < c.n_agents);
    // L1: lane 0 k1, lane 1 key_reset, lane 2+t split(key, n_types)[t]
    const Key L1 = split_key(key, l < 2 ? 2 : nTy, l < 2 ? l : l - 2, part);
    StepKeys o;
    o.key = key;
    o.next_master = nm;
    o.k1 = Key{(u32)rdl((i32)L1.a, 0), (u32)rdl((i32)L1.b, 0)};
    o.key_reset = Key{(u32)rdl((i32)L1.a, 1), (u32)rdl((i32)L1.b, 1)};
    if (two) {
        const Key P2 = from_lane(L1, agent_lane ? 2 + t : 0);
        const Key L2 = split_key(P2, agent_lane ? type_n_agents(c, t) : 2, agent_lane ? i : 1, part);
        // L3: lane 0 sub = split(sk)[1]; lane 32 + ag split(k_ag)[0]; lane 48 + ag split(k_ag)[1]
        const Key L3 = split_key(L2, 2, ((l == 0) | hi_lane) ? 1 : 0, part);
        // L4: lanes < A random_bits(sub, A)[l]; agent lanes random_bits(their key, 1)[0]
        const Key sub = from_lane(L3, 0);
        const u32 bits = random_bits(l < A ? sub : L3, 1, l < A ? l : 0, part);
        o.shuffle_bits = bits;
        const u32 hb = bits, lb = (u32)__builtin_amdgcn_ds_bpermute(((l + 16) & 63) << 2, (i32)bits);
        const i32 na = agent_lane ? type_action_hi(c, t, MD) : 1;
        const u32 span = na <= 0 ? 1u : (u32)na;
        u32 mult = 65536u % span;
        mult = (mult * mult) % span;
        o.acts = (i32)(((hb % span) * mult + (lb % span)) % span);
        return o;
    }
    // L2: lane 0 sk = split(k1)[1]; agent lanes: split(sub_t, n_agents_t)[i]
    const Key P2 = from_lane(L1, agent_lane ? 2 + t : 0);
    const Key L2 = split_key(P2, agent_lane ? type_n_agents(c, t) : 2, agent_lane ? i : 1, part);
    // L3: lane 0 sub = split(sk)[1]; agent lanes: randint's two keys
    const Key L3a = split_key(L2, 2, l == 0 ? 1 : 0, part);
    const Key L3b = split_key(L2, 2, 1, part);
    // L4: lanes < A: random_bits(sub, A)[l]; agent lanes: the two randint words
    const Key sub = from_lane(L3a, 0);
    o.shuffle_bits = random_bits(sub, A > 0 ? A : 1, l < A ? l : 0, part);
    const u32 hb = random_bits(L3a, 1, 0, part), lb = random_bits(L3b, 1, 0, part);
    const i32 na = agent_lane ? type_action_hi(c, t, MD) : 1;
    const u32 span = na <= 0 ? 1u : (u32)na;  // randint(key, 0, n_actions)
    u32 mult = 65536u % span;
    mult = (mult * mult) % span;
    o.acts = (i32)(((hb % span) * mult + (lb % span)) % span);
    return o;
}

// Rollout steps' keys in batches (k_env_rollout; partitionable keys, <= 3 agents, <= 8 action
// rows, <= 6 agent types, agents + action rows <= 10).  Speed_test's actions are random, so step t + j's keys depend only on
// the master-key chain: up to KB_STEPS steps are derived at once, step j in lanes 16j..16j+15
// (ll = lane & 15: the lanes of step_keys' two-lane layout, folded into 16: ll 0 / 1 / 2 + t the
// first level, agent ag's two randint words in ll 8 + ag and 12 + ag, shuffle words in ll < A).
// The master chain (split(m_j, n + 1)[0]) and the env keys (split(m_j, n + 1)[e + 1]) take one
// level per step, then the four levels below the env key run for all the batch's steps at once:
// 4 + 4 dependent threefry levels per 4 steps instead of 5 per step.  Bit-identical to step_keys.
// Output per step j in LDS, kb[j * kb_words(c) + ...]: key (2), k1 (2), key_reset (2), the
// agents' actions (n_agents), the shuffle words (A).
#define KB_STEPS 4
__host__ __device__ inline bool kb_ok(const hftlob_env_cfg& c) {  // (a step's row: one word per lane of its 16)
    return c.prng_partitionable && c.n_agents <= 3 && c.n_action_msgs <= 8 && c.n_types <= 6 &&
           6 + c.n_agents + c.n_action_msgs <= 16;
}
__host__ __device__ inline int kb_words(const hftlob_env_cfg& c) { return 6 + c.n_agents + c.n_action_msgs; }
// LDS carve-up of one env's workgroup (words): [agent rows (C+A)*8][action extras][book: asks 6nO,
// bids 6nO, trades 8nT, pad 256][key batches].  The agent rows can live IN the trade log instead:
// it is free from the step's start until trades_fill, which then runs once the rows are read.
// (Speed_test's [5,5] agents: 60 rows, 1.9 KB less per env, 16 envs per CU instead of 14.)
// The rows may span two message chunks (C + A <= 128): the second chunk's agent rows are read into
// its registers with the first chunk's, before trades_fill.  They may run past the trade log into
// the pad's over-read area and filter words (both unused until chunk 0's rows are read), not into
// its scratch row (filter_rows' scratch): (C + A) * 8 <= 8 nT + 192 words.  (Speed_test's [10, 10]
// agents: 120 rows at nT = 100.)
__host__ __device__ inline bool rows_in_trades(const hftlob_env_cfg& c, int nT) {
    const int ar = c.n_cancel_msgs + c.n_action_msgs;
    return ar <= 128 && 8 * ar <= 8 * nT + 192;
}
struct LdsMap {
    int rows, axs, book, kb, words;  // word offsets, total words
};
// alias: the rows-in-trades layout (a separate kernel instantiation, RA, launched only where it
// raises the envs a CU holds: use_rows_alias; the other kernels keep the rows' own region at 0)
__host__ __device__ inline LdsMap lds_map(const hftlob_env_cfg& c, int nO, int nT, bool alias) {
    LdsMap m;
    const int rw = alias ? 0 : (c.n_cancel_msgs + c.n_action_msgs) * 8;
    m.axs = rw;
    m.book = rw + ((c.n_agents * 6 + 3) & ~3);
    m.rows = alias ? m.book + 12 * nO : 0;  // (the trade log)
    m.kb = m.book + 12 * nO + 8 * nT + 256;
    m.words = m.kb + (kb_ok(c) ? KB_STEPS * kb_words(c) : 0);
    return m;
}
template <bool MD>
DEV void step_keys_batch(const hftlob_env_cfg& c, int n_env, int e, Key& mk, int nb, i32* kb) {
    const bool part = true;
    const int l = lane_id(), ll = l & 15, j = l >> 4, nTy = c.n_types, A = c.n_action_msgs, KW = kb_words(c);
    // the chain: level q gives m_{q+1} (lane 0) and step q's env key (lane 1)
    i32 ka = 0, kb2 = 0;  // lane 16j: step j's env key
#pragma unroll 1
    for (int q = 0; q < nb; ++q) {
        const Key v = split_key(mk, n_env + 1, l == 1 ? e + 1 : 0, part);
        ka = wlane(ka, rdl((i32)v.a, 1), 16 * q);
        kb2 = wlane(kb2, rdl((i32)v.b, 1), 16 * q);
        mk = Key{(u32)rdl((i32)v.a, 0), (u32)rdl((i32)v.b, 0)};
    }
    const int b0 = l & ~15;  // this lane's step block
    const Key key{(u32)__builtin_amdgcn_ds_bpermute(b0 << 2, ka), (u32)__builtin_amdgcn_ds_bpermute(b0 << 2, kb2)};
    const bool hi_lane = ll >= 12;
    const int ag = ll - (hi_lane ? 12 : 8);
    int t = 0, i = 0;
    agent_of_lane(c, ag < 0 ? 0 : ag, t, i);
    const bool agent_lane = (ll >= 8) & (ag >= 0) & (ag < c.n_agents);
    const Key L1 = split_key(key, ll < 2 ? 2 : nTy, ll < 2 ? ll : ll - 2, part);
    const Key P2 = from_lane(L1, b0 + (agent_lane ? 2 + t : 0));
    const Key L2 = split_key(P2, agent_lane ? type_n_agents(c, t) : 2, agent_lane ? i : 1, part);
    const Key L3 = split_key(L2, 2, ((ll == 0) | hi_lane) ? 1 : 0, part);
    const Key sub = from_lane(L3, b0);
    const u32 bits = random_bits(ll < A ? sub : L3, 1, ll < A ? ll : 0, part);
    const u32 hb = bits, lb = (u32)__builtin_amdgcn_ds_bpermute(((l + 4) & 63) << 2, (i32)bits);
    const i32 na = agent_lane ? type_action_hi(c, t, MD) : 1;
    const u32 span = na <= 0 ? 1u : (u32)na;
    u32 mult = 65536u % span;
    mult = (mult * mult) % span;
    const i32 act = (i32)(((hb % span) * mult + (lb % span)) % span);
    // LDS: lane 16j + w writes word w of step j's row: 0..5 keys (from lanes ll 0 / 1 of L1 and
    // the block's env key), 6 + ag the actions (ll 8 + ag), 6 + n_agents + r the shuffle words
    // (ll 2 / 3: k1 = L1 of ll 0; ll 4 / 5: key_reset = L1 of ll 1)
    const i32 l1a = __builtin_amdgcn_ds_bpermute((b0 + ((ll >> 2) & 1)) << 2, (i32)L1.a);
    const i32 l1b = __builtin_amdgcn_ds_bpermute((b0 + ((ll >> 2) & 1)) << 2, (i32)L1.b);
    const i32 ac = __builtin_amdgcn_ds_bpermute((b0 + 8 + (ll >= 6 ? ll - 6 : 0)) << 2, act);
    const i32 sh = __builtin_amdgcn_ds_bpermute((b0 + (ll >= 6 + c.n_agents ? ll - 6 - c.n_agents : 0)) << 2, (i32)bits);
    i32 w = ll == 0 ? (i32)key.a : (ll == 1 ? (i32)key.b : ((ll & 1) ? l1b : l1a));
    w = ll >= 6 + c.n_agents ? sh : (ll >= 6 ? ac : w);
    if ((j < nb) & (ll < KW)) kb[j * KW + ll] = w;
    wave_sync();
}
// step j's keys from the batch row (as step_keys would derive them)
DEV StepKeys load_keys(const hftlob_env_cfg& c, const i32* row) {
    const int l = lane_id(), na = c.n_agents, A = c.n_action_msgs;
    StepKeys o;
    o.key = Key{(u32)uni(row[0]), (u32)uni(row[1])};
    o.k1 = Key{(u32)uni(row[2]), (u32)uni(row[3])};
    o.key_reset = Key{(u32)uni(row[4]), (u32)uni(row[5])};
    o.next_master = Key{0u, 0u};
    const int ag = l - 32;
    o.acts = ((ag >= 0) & (ag < na)) ? row[6 + (ag < 0 ? 0 : ag)] : 0;
    o.shuffle_bits = l < A ? (u32)row[6 + na + (l < A ? l : 0)] : 0u;
    return o;
}

// BaseLOBEnv.get_data_messages, fixed_time (base_env.py:358-367): a data row
// whose time_s >= the episode end time becomes [0 x 6, time_s, time_ns]
DEV void fixed_time_mask(int4& x, int4& y, i32 t_end) {
    if (y.z >= t_end) {
        x = make_int4(0, 0, 0, 0);
        y.x = 0;
        y.y = 0;
    }
}

// world debug_mode (marl_env.py:645-656): get_L2_state of the stepped books
// (JaxOrderBookArrays.py:1231-1264) and the step's trade log.  Ten ascending-unique passes per
// side: level k = the least key above level k-1 (the whole side for k = 0), a missing level
// takes jnp.unique's fill; volumes get_volume_at_price at the level's (replaced) price.
// bid key -p (an empty row's -1 is the level 1), fill 1, then -1 -> -maxint; ask key p with
// -1 -> maxint, fill -1, then -1 -> maxint.  Negative volumes read 0.
template <bool BID, int S>
DEV i32 l2_side(const Side<S>& s, int R, const Valid<S>& V, i32 maxint, i32 outv) {
    const int l = lane_id();
    i32 x[S], q[S];
    ldcol(s.t, R, FQ, q);
#pragma unroll
    for (int r = 0; r < S; ++r) x[r] = BID ? wmul(-1, s.pc[r]) : (s.pc[r] == -1 ? maxint : s.pc[r]);
    i32 prev = 0;
    for (int k = 0; k < HFTLOB_L2_LEVELS; ++k) {
        i32 m = INT_MAX;
        lmask any = 0;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const bool ok = V.v[r] && (k == 0 || x[r] > prev);
            m = imin_(m, ok ? x[r] : INT_MAX);
            any |= bal(ok);
        }
        i32 lv = wave_min(m);
        if (any == 0ull) lv = BID ? 1 : -1;
        else prev = lv;
        i32 p = BID ? wmul(-1, lv) : lv;
        p = p == -1 ? (BID ? wsub(0, maxint) : maxint) : p;
        i32 v = 0;
#pragma unroll
        for (int r = 0; r < S; ++r) v = wadd(v, (V.v[r] && s.pc[r] == p) ? q[r] : 0);
        const i32 vol = imax_(wave_sum(v), 0);
        const int c = k * 4 + (BID ? 2 : 0);
        outv = l == c ? p : (l == c + 1 ? vol : outv);
    }
    return outv;
}
template <int S> DEV void write_debug(const Book<S>& B, i32* dst) {
    const int l = lane_id(), R = B.c.nO;
    i32 v = 0;
    v = l2_side<false>(B.a, R, B.vs, B.c.maxint, v);
    v = l2_side<true>(B.b, R, B.vs, B.c.maxint, v);
    if (l < 4 * HFTLOB_L2_LEVELS) dst[l] = v;
    store_trades(B.tr, dst + 4 * HFTLOB_L2_LEVELS, B.vt);
}

// ====================================================== K2: fused env step
// MARLEnv.step — marl_env.py:775-804 (step_env :211-709, auto-reset select)
#define MAX_AGENT_ROWS 128
// NFIX > 0: nOrders == nTrades == NFIX known at compile time (the reference's
// 100/100 default), which folds the slot-validity masks away.
template <int S, int NFIX, bool RC, bool RA = false, bool QUIET = false, int PK = -1>
// RC: cancel_mode 2/3 (the random cancel fallback of the engine).  RA: the agent rows live in the
// trade log (lds_map).  QUIET: a step whose outputs are never emitted (emit = false at compile
// time: k_env_rollout's per_step = 0 steps before the last, whose copy of the step body then holds
// no observation or reward-value code).  PK: 1 = the step's keys always come from a key-batch row
// (pre_keys, k_env_rollout's KB = 1), 0 = never, -1 = as pre_keys is given.
// master: Speed_test rollout mode — the env's step key is split(mk, n_env + 1)[e + 1],
// actions are sampled here (hftlob_sample_actions) and written to actions_io if it is not
// NULL; mk becomes split(mk)[0].  Otherwise keys / actions_io are the inputs.  (mk is a
// reference, not a pointer: an address-taken local would live in scratch memory.)
// key_n / ek: the env count of the step-key split and this env's index in it;
// e: this env's record / output index.
// emit (wave-uniform): the step's outputs are wanted.  k_env_rollout with per_step = 0 passes
// false on every step but the last: Speed_test's scan keeps only the state (its jitted body
// returns `_, state, _, _, _`, so XLA drops the observations and the reward values, which feed no
// state), and each step's outputs would be overwritten by the next.  Then the observations, the
// reward values (not the PnL / cash / inventory / execution statistics the agent states carry),
// the dones and the output stores are skipped; the state is bit-identical either way.
DEV bool env_step_dev(const hftlob_env_cfg& c, int key_n, int ek, int e, const u32* __restrict__ keys, bool master,
                      Key& mk,
                      i32* __restrict__ actions_io, const i32* __restrict__ msg_data,
                      const i32* __restrict__ init_states, i32* __restrict__ state, float* __restrict__ obs_out,
                      float* __restrict__ rew_out, u8* __restrict__ done_all_out, u8* __restrict__ dones_out,
                      i32* __restrict__ info_out, i32* __restrict__ obs_raw_out, i32* __restrict__ msgs_out,
                      i32* __restrict__ debug_out, i32* lds, bool resident, bool keep, u32& fl_carry,
                      const i32* pre_keys = nullptr, bool emit_rt = true) {
    const bool emit = !QUIET && emit_rt;
    STAMP(t_start);
#ifdef HFTLOB_STAMPS
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz: the in-kernel clock
#endif
    const int l = lane_id();
    const int M = c.n_msgs, D = c.n_data_msg, A = c.n_action_msgs, C = c.n_cancel_msgs;
    i32* rec = state + (size_t)e * c.rec_words;
    // LDS: [agent rows (C+A)*8][action extras n_agents*6, 16B-padded][book]
    Book<S> B;
    B.c = lobcfg(c.lob);
    if (NFIX > 0) { B.c.nO = NFIX; B.c.nT = NFIX; }
    const int R = B.c.nO;
    const LdsMap LM = lds_map(c, B.c.nO, B.c.nT, RA);
    i32* rows = lds + LM.rows;
    i32* axs = lds + LM.axs;
    book_bind(B, lds + LM.book);
    SideRows<S> fa, fb;  // issue the book's HBM loads first; they land while the keys are derived
    if (!resident) {
        fetch_side(fa, rec + c.off_asks, B.vs);
        fetch_side(fb, rec + c.off_bids, B.vs);
    }
    // the agent states (<= 64 words: one per lane), loaded with the book: the agent and reward
    // phases read them with v_readlane instead of waiting on scalar loads per agent
    const int naw = c.rec_words - c.off_agents;
    const bool agw_pre = naw <= 64;
    const i32 agw = (agw_pre & (l < naw)) ? rec[c.off_agents + l] : 0;
    // (pre_keys: this step's row of a k_env_rollout key batch, step_keys_batch)
    const bool batched = PK == 1 || (PK < 0 && pre_keys);
    const StepKeys SK = batched ? load_keys(c, pre_keys) : step_keys<NFIX == 0>(c, key_n, ek, keys, master, mk);
    if (master && !batched) mk = SK.next_master;
    const Key key_reset = SK.key_reset;
    if (RC) {  // the scan's key: k1, or split(k1)[0] after the shuffle split (marl_env.py:293-294,349-351)
        B.ek = c.shuffle_action_messages ? split_key(SK.k1, 2, 0, c.prng_partitionable) : SK.k1;
        B.nmsg = M;
        B.part = c.prng_partitionable;
    }
    SUBSTAMP(t_keys);
    // loaded / world scalars (wave-uniform)
    const i32* Lr = rec + c.off_loaded;
    const i32* Wr = rec + c.off_world;
    const i32 ld_t0 = Lr[LD_T0], win = Lr[LD_WIN], max_steps = Lr[LD_MAXS], start_index = Lr[LD_START],
              step = Lr[LD_STEP];
    const i32 wt0 = Wr[W_T0], wt1 = Wr[W_T1], oidc = Wr[W_OIDC];
    const float wmid = bitf(Wr[W_MID]);
    const i32 old_last_ba = rec[c.off_best_asks + (M - 1) * 2], old_last_bb = rec[c.off_best_bids + (M - 1) * 2];
    bool excl_any = false, excl_cfg = false;
    for (int t = 0; t < c.n_types; ++t) {
        const bool ex = c.types[t].kind == HFTLOB_AGENT_MM && c.types[t].exclude_extreme_spreads;
        excl_cfg |= ex;
        if (emit && ex) {
            bool any = false;
            for (int m = l; m < M; m += 64) {
                const i32 pa = rec[c.off_best_asks + m * 2], pb = rec[c.off_best_bids + m * 2];
                any |= (i2f(wsub(pa, pb)) / (i2f(wadd(pa, pb)) / 2.0f)) > 0.1f;
            }
            excl_any = ballot(any) != 0ull;
        }
    }
    // the step's best-quote arrays go to the record when they can be read: always in k_env_step, on a
    // persistent rollout's last step, and whenever an MM type excludes extreme spreads (its reward
    // reads the previous step's arrays).  Otherwise the next step reads only their last row (the
    // old best quotes above), which the step stores alone; the step after that overwrites the rest.
    const bool store_best = !keep | excl_cfg;
    // the data window (BaseLOBEnv.get_data_messages, base_env.py:339-369); its
    // first chunk is fetched now, ahead of the agent phase
    i32 dstart = wadd(start_index, wmul(D, step));
    dstart = imax_(0, imin_(dstart, c.n_data_rows - D));  // dynamic_slice clamping
    // fixed_time: rows at or after init_time[0] + episode_time keep only their time (base_env.py:358-367)
    const bool ftime = NFIX == 0 && c.ep_type == 1;  // the 100/100 kernel is launched for fixed_steps only
    const i32 t_end = wadd(ld_t0, c.episode_time);
    int4 px = make_int4(0, 0, 0, 0), py = px;
    if ((l >= C + A) & (l < M)) {
        const i32* g = msg_data + (size_t)(dstart + l - (C + A)) * 8;
        px = reinterpret_cast<const int4*>(g)[0];
        py = reinterpret_cast<const int4*>(g)[1];
        if (ftime) fixed_time_mask(px, py, t_end);
    }
    if (resident) {  // the book flags as the previous step left them (the cached best quotes are not kept)
        relink_side(B.a, R, B.vs);
        relink_side(B.b, R, B.vs);
        B.fl = fl_carry | F_STALE_A | F_STALE_B | STALE_ANY;
    } else {
        B.fl = commit_side<true>(B.a, fa, R, B.vs) | commit_side<false>(B.b, fb, R, B.vs) | F_STALE_A | F_STALE_B | STALE_ANY;
        B.fl |= slow_bit(B.fl);
    }
    SUBSTAMP(t_load);

    // ---- (C) agent messages -> LDS rows [cancels C][actions A]
#ifdef HFTLOB_STAMPS
    unsigned long long acc_act = 0, acc_cnl = 0, acc_flt = 0, acc_mmr = 0, acc_exr = 0, acc_obs = 0;
#endif
    {
        int ag = 0, arow = C, crow = 0, aw = 0;
        const i32* st = rec + c.off_agents;
        for (int t = 0; t < c.n_types; ++t) {
            const hftlob_agent_type_cfg& tc = c.types[t];
            for (int i = 0; i < tc.n_agents; ++i, ++ag) {
                const i32 tid = wsub(tc.trader_id0, i);
                const int w = tc.action_width;
                i32* aio = actions_io ? actions_io + (size_t)e * c.action_words + aw : nullptr;
                aw += w;
                i32 act, av[4] = {0, 0, 0, 0};
                if (NFIX > 0 || w == 1) {  // the 100/100 kernel is launched for Discrete spaces only
                    if (master) {  // Speed_test.py:166-177, sampled by step_keys
                        act = rdl(SK.acts, 32 + ag);
                        if (aio && l == 0) aio[0] = act;
                    } else {
                        act = aio[0];
                    }
                    av[0] = act;
                } else {  // MultiDiscrete: lane j < w draws word j (spaces.py:57-65)
                    i32 v = 0;
                    if (master) {
                        const bool part = c.prng_partitionable;
                        const Key ka = split_key(split_key(SK.key, c.n_types, t, part), tc.n_agents, i, part);
                        v = randint_vec(ka, w, l < w ? l : 0, 0, action_hi(tc), part);
                        if (aio && l < w) aio[l] = v;
                    } else if (l < w) {
                        v = aio[l];
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) av[j] = rdl(v, j);
                    act = av[0];
                }
                i32 s4[4];
                {
                    const int b = (int)(st - (rec + c.off_agents));
#pragma unroll
                    for (int k = 0; k < 4; ++k) s4[k] = agw_pre ? rdl(agw, b + k) : st[k];
                }
                ActX x{0, 0, 0, 0, 0, 0};
                SUBSTAMP(ta0);
#if defined(HFTLOB_KO_ACT) || defined(HFTLOB_KO_CNL)  // timing knockout builds only (wrong results)
                for (int k = 0; k < tc.n_msgs; ++k) {
#ifndef HFTLOB_KO_ACT
                    if (k < tc.n_action_msgs) continue;
#endif
#ifndef HFTLOB_KO_CNL
                    if (k >= tc.n_action_msgs) continue;
#endif
                    put_row(rows, k < tc.n_action_msgs ? arow + k : crow + k - tc.n_action_msgs, 0, 0, 0, 0, 0, 0, 0, 0);
                }
#endif
#ifdef HFTLOB_DUP_AGENT  // timing builds only: the agent's action (bit 0) / cancel (bit 1) rows computed twice
                i32 z_ = 0;     // (an opaque zero keeps the second pass from being hoisted or merged)
                asm volatile("s_mov_b32 %0, 0" : "=s"(z_));
                for (int rep = 0; rep < 2; ++rep) {
                const i32 tid_r = tid ^ (rep * z_), act_r = act ^ (rep * z_), ba_r = old_last_ba ^ (rep * z_);
                const bool do_act = rep == 0 || (HFTLOB_DUP_AGENT & 1), do_cnl = rep == 0 || (HFTLOB_DUP_AGENT & 2);
#else
                {
                const i32 tid_r = tid, act_r = act, ba_r = old_last_ba;
                constexpr bool do_act = true, do_cnl = true;
#endif
                if (tc.kind == HFTLOB_AGENT_MM) {
#ifndef HFTLOB_KO_ACT
                    if (!do_act) {
                    } else if (tc.action_space == HFTLOB_MM_ACT_DIRECTIONAL)
                        mm_directional(c, tc, tid_r, act_r, wt0, wt1, ba_r, old_last_bb, rows, arow, x);
                    else if (tc.action_space == HFTLOB_MM_ACT_FIXED_QUANTS)
                        mm_fixed_quant(c, tc, B, s4, tid_r, act_r, wt0, wt1, ba_r, old_last_bb, rows, arow, x);
                    else
                        mm_other_actions(c, tc, B, s4, tid_r, act_r, wt0, wt1, ba_r, old_last_bb, step, ld_t0, rows,
                                         arow, x);
#endif
                    STAMP_ACC(acc_act, ta0);
                    SUBSTAMP(ta1);
                    const int sz = tc.n_msgs / 4;
#ifndef HFTLOB_KO_CNL
                    if (do_cnl) {
                        cancel_rows(B.b, R, B.vs, tid_r, sz, 1, wt0, wt1, rows, crow);
                        cancel_rows(B.a, R, B.vs, tid_r, sz, -1, wt0, wt1, rows, crow + sz);
                    }
#endif
                    STAMP_ACC(acc_cnl, ta1);
                } else {
#ifndef HFTLOB_KO_ACT
                    if (!do_act) {
                    } else if (NFIX == 0 && tc.action_space == HFTLOB_EXE_ACT_FIXED_PRICES)
                        exe_fixed_prices(c, tc, rec, s4, tid_r, av, wt0, wt1, rows, arow);
                    else
                        exe_fqc(c, tc, s4, tid_r, act_r, wt0, wt1, ba_r, old_last_bb, step, max_steps, rows, arow);
#endif
                    STAMP_ACC(acc_act, ta0);
                    SUBSTAMP(ta1);
#ifndef HFTLOB_KO_CNL
                    const i32 sell = s4[3];
                    if (do_cnl)
                        cancel_rows(sell ? B.a : B.b, R, B.vs, tid_r, tc.n_msgs / 2, wsub(1, wmul(sell, 2)), wt0, wt1,
                                    rows, crow);
#endif
                    STAMP_ACC(acc_cnl, ta1);
                }
                }
                SUBSTAMP(ta2);
                {
                    const i32 xv[6] = {x.bid_price, x.ask_price, x.bid_dist, x.ask_dist, x.bid_quant, x.ask_quant};
                    i32 v = 0;
#pragma unroll
                    for (int k = 0; k < 6; ++k) if (l == k) v = xv[k];
                    if (l < 6) axs[ag * 6 + l] = v;
                }
#ifndef HFTLOB_KO_FILTER  // timing knockout builds only (wrong results)
                if (tc.n_action_msgs == 2) filter_rows<2>(rows, arow, crow, B.a.scr);
                else if (tc.n_action_msgs == 4) filter_rows<4>(rows, arow, crow, B.a.scr);
                else if (NFIX == 0 && tc.n_action_msgs == 3) filter_rows<3>(rows, arow, crow, B.a.scr);  // fixed_prices
                else filter_rows<1>(rows, arow, crow, B.a.scr);
#endif
                STAMP_ACC(acc_flt, ta2);
                arow += tc.n_action_msgs;
                crow += tc.n_msgs - tc.n_action_msgs;
                st += agent_words(tc);
            }
        }
    }
    wave_sync();
    SUBSTAMP(t_rows);
    // order ids (counter - j) and the action-row permutation (lane j = action row j)
    {
        i32 f[8];
        const bool act_lane = l < A;
        if (act_lane) {
#pragma unroll
            for (int k = 0; k < 8; ++k) f[k] = rows[(C + l) * 8 + k];
            f[4] = wsub(oidc, l);
        }
        int dest = l;
        if (c.shuffle_action_messages && A >= 2) {
            const u32 bits = SK.shuffle_bits;
            int rank = 0;
            for (int j = 0; j < A; ++j) {
                const u32 bj = (u32)rdl((i32)bits, j);
                rank += (bj < bits) || (bj == bits && j < l);
            }
            dest = rank;
        }
        wave_sync();
        if (act_lane) {
#pragma unroll
            for (int k = 0; k < 8; ++k) rows[(C + dest) * 8 + k] = f[k];
        }
        wave_sync();
    }

    STAMP(t_agents);
    // ---- (B)+(D) stream the combined messages through the book, 64 per chunk
    if (!RA) trades_fill(B.tr, B.vt, -1);
    B.ntr = 0;
    const int AR = C + A;
    bool abort_any = false;
    i32 prev_a = -1, prev_b = -1;
    float mid_acc = 0.0f, pa_acc = 0.0f, pb_acc = 0.0f;
    i32 last_p_a = 0, last_p_b = 0, last_t0 = 0, last_t1 = 0;
    int4 nx = px, ny = py;  // the chunk's data rows, loaded one chunk ahead (chunk 0's at kernel start)
    for (int base = 0; base < M; base += 64) {
        const int row = base + l;
        int4 x = nx, y = ny;
        if (RA ? (base == 0) & (row < AR) : row < AR) {  // (RA: chunk 1's agent rows came with chunk 0's)
            x = reinterpret_cast<const int4*>(rows + row * 8)[0];
            y = reinterpret_cast<const int4*>(rows + row * 8)[1];
        } else if (ftime && base > 0 && row >= AR) {
            fixed_time_mask(x, y, t_end);
        }
        if (msgs_out && row < M) {  // the combined message row as the book receives it ("messages" obs)
            int4* mo = reinterpret_cast<int4*>(msgs_out + ((size_t)e * M + row) * 8);
            mo[0] = x;
            mo[1] = y;
        }
        nx = make_int4(0, 0, 0, 0);
        ny = nx;
        if ((row + 64 >= AR) & (row + 64 < M)) {  // the next chunk's loads land while this one runs
            const i32* g = msg_data + (size_t)(dstart + row + 64 - AR) * 8;
            nx = reinterpret_cast<const int4*>(g)[0];
            ny = reinterpret_cast<const int4*>(g)[1];
        }
        if (RA && (base == 0)) {  // the step's trade log starts all -1: reset once the agent rows, which
            if (row + 64 < AR) {  // live in it, are read (chunk 1's into its registers; a wave's LDS
                nx = reinterpret_cast<const int4*>(rows + (row + 64) * 8)[0];  // operations run in order)
                ny = reinterpret_cast<const int4*>(rows + (row + 64) * 8)[1];
            }
            wave_sync();
            trades_fill(B.tr, B.vt, -1);
        }
        decode_msgs(B.c, x, y);
        i32 rpa = 0, rqa = 0, rpb = 0, rqb = 0;
        const int cnt = uni(imin_(64, M - base));  // SGPR: the loop test stays on the scalar unit
        run_chunk<RC>(B, x, y, cnt, base, rpa, rqa, rpb, rqb);
        // abort flag on raw quotes; _ffill_best_prices (marl_env.py:723-749) for the chunk
        abort_any |= bal((l < cnt) & ((rpa == -1) | (rpb == -1))) != 0ull;
        i32 pa = rpa, pb = rpb;
        if ((base == 0) & (l == 0)) {
            pa = pa == -1 ? old_last_ba : pa;
            pb = pb == -1 ? old_last_bb : pb;
        }
        const i32 caq = rpa == -1 ? 0 : rqa, cbq = rpb == -1 ? 0 : rqb;
        const i32 cap = ffill(pa, prev_a), cbp = ffill(pb, prev_b);
        prev_a = rdl(cap, cnt - 1);
        prev_b = rdl(cbp, cnt - 1);
        if ((row < M) & (store_best | (row == M - 1))) {  // (row M - 1: the one the next step reads)
            reinterpret_cast<int2*>(rec + c.off_best_asks)[row] = make_int2(cap, caq);
            reinterpret_cast<int2*>(rec + c.off_best_bids)[row] = make_int2(cbp, cbq);
        }
        if (row < M) {
            const float mf = i2f(wadd(cbp, cap)) / 2.0f;
            mid_acc = base == 0 ? mf : mid_acc + mf;
            if (info_out) {  // (the info's average quotes only)
                pa_acc = base == 0 ? i2f(cap) : pa_acc + i2f(cap);
                pb_acc = base == 0 ? i2f(cbp) : pb_acc + i2f(cbp);
            }
        }
        if (base + 64 >= M) {  // final time = last combined row's (s, ns)
            last_t0 = rdl(y.z, cnt - 1);
            last_t1 = rdl(y.w, cnt - 1);
        }
    }
    last_p_a = prev_a;
    last_p_b = prev_b;
    StepCtx X;
    X.avg_mid = wave_fsum(mid_acc) / (float)M;
    X.last_ba = last_p_a; X.last_bb = last_p_b;
    X.last_mid = i2f(wadd(last_p_b, last_p_a)) / 2.0f;
    X.wmid = wmid;
    X.old_last_ba = old_last_ba; X.old_last_bb = old_last_bb;
    X.init0 = ld_t0; X.step = step;
    X.ep_done = wsub(wsub(max_steps, step), 1) <= 1;
    const bool all = X.ep_done;

    STAMP(t_book);
    // ---- (E) rewards, (G) agent states, (K) observations
    WorldView wv;
    wv.best_ask_p = last_p_a; wv.best_bid_p = last_p_b;
    wv.vol_a = wv.vol_b = 0;
    if (emit) { wv.vol_a = side_volume(B.a, R, B.vs); wv.vol_b = side_volume(B.b, R, B.vs); }
    if (debug_out) write_debug(B, debug_out + (size_t)e * HFTLOB_DEBUG_WORDS(B.c.nT));  // before store / reset
    // the book is final: store it now (frees its registers for the rewards).  Not when the
    // auto-reset below rewrites the record anyway, nor while the wave's next step (keep,
    // k_env_rollout) takes the book and trade log from LDS as they are
    if (keep) fl_carry = B.fl;
    if (!all & !keep) {
        store_side(B.a, rec + c.off_asks, R, B.vs);
        store_side(B.b, rec + c.off_bids, R, B.vs);
        store_trades(B.tr, rec + c.off_trades, B.vt);
    }
    wv.step = wadd(step, 1); wv.max_steps = max_steps; wv.mid = X.last_mid;
    wv.t0 = last_t0; wv.t1 = last_t1; wv.it0 = ld_t0; wv.it1 = Lr[LD_T1];
    const float dt = i2f(last_t0) + i2f(last_t1) / 1e9f - i2f(wt0) - i2f(wt1) / 1e9f;  // marl_env.py:496
    wv.dt = dt;
    i32* info = info_out ? info_out + (size_t)e * c.info_words : nullptr;
    if (emit | !all) {  // (an unemitted episode end: the auto-reset below replaces every agent state)
        // the step's trade log as the rewards read it, loaded once for every agent
        TradeView<S> TV;
        {
            const i32 ovr0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            trade_view(B, TV, false, -1, ovr0);
        }
        int ag = 0;
        i32* st = rec + c.off_agents;
        for (int t = 0; t < c.n_types; ++t) {
            const hftlob_agent_type_cfg& tc = c.types[t];
            for (int i = 0; i < tc.n_agents; ++i, ++ag) {
                const i32 tid = wsub(tc.trader_id0, i);
                const int nw = agent_words(tc);
                i32 s[13];
                {
                    const int b = (int)(st - (rec + c.off_agents));
                    for (int k = 0; k < 13; ++k) s[k] = k < nw ? (agw_pre ? rdl(agw, b + k) : st[k]) : 0;
                }
                i32 d = 0;
                float rew;
                i32 iw[HFTLOB_INFO_AGENT_WORDS];
                for (int k = 0; k < HFTLOB_INFO_AGENT_WORDS; ++k) iw[k] = 0;
                ActX ax1;
                ax1.bid_price = uni(axs[ag * 6 + 0]); ax1.ask_price = uni(axs[ag * 6 + 1]);
                ax1.bid_dist = uni(axs[ag * 6 + 2]); ax1.ask_dist = uni(axs[ag * 6 + 3]);
                ax1.bid_quant = uni(axs[ag * 6 + 4]); ax1.ask_quant = uni(axs[ag * 6 + 5]);
                SUBSTAMP(tr0);
                if (tc.kind == HFTLOB_AGENT_MM) {
                    MMRew R;
#if defined(HFTLOB_KO_REWARD) || defined(HFTLOB_KO_MM_REWARD)  // timing knockout builds only (wrong results)
                    memset(&R, 0, sizeof R);
#else
                    mm_reward(c, tc, B, X, s, tid, excl_any, TV, R, emit);
#endif
                    STAMP_ACC(acc_mmr, tr0);
                    const float tot = bitf(s[3]) + R.PnL;
                    s[0] = ax1.bid_dist; s[1] = ax1.ask_dist; s[2] = R.end_inventory; s[3] = fbit(tot);
                    s[4] = fbit(R.cash);
                    rew = R.reward / tc.reward_scaling_quo;
                    iw[0] = fbit(R.reward); iw[1] = fbit(R.reward_pv); iw[2] = fbit(R.reward_spooner);
                    iw[3] = fbit(R.end_of_ep_pv); iw[4] = fbit(R.reward_spooner_damped);
                    iw[5] = fbit(R.reward_spooner_asym_damped); iw[6] = fbit(R.reward_spooner_asym_damped2);
                    iw[7] = fbit(R.reward_delta_pv); iw[8] = fbit(tot); iw[9] = 0; iw[10] = s[2];
                    iw[11] = fbit(R.delta_mid); iw[12] = fbit(R.market_share); iw[13] = fbit(R.buyPnL);
                    iw[14] = R.forced_unwind; iw[15] = fbit(R.invPnL); iw[16] = ax1.bid_price;
                    iw[17] = ax1.ask_price; iw[18] = ax1.bid_dist; iw[19] = ax1.ask_dist;
                    iw[20] = ax1.ask_quant; iw[21] = ax1.bid_quant; iw[22] = fbit(R.sellPnL);
                    iw[23] = fbit(R.inventoryValue);
                } else {
                    EXRew R;
#if defined(HFTLOB_KO_REWARD) || defined(HFTLOB_KO_EXE_REWARD)
                    memset(&R, 0, sizeof R);
#else
                    exe_reward(c, tc, B, X, s, tid, TV, R, emit);
#endif
                    STAMP_ACC(acc_exr, tr0);
                    s[2] = wadd(s[2], R.agentQuant);
                    s[4] = fbit(R.p_vwap);
                    s[5] = fbit(bitf(s[5]) + i2f(R.qp_agent));
                    s[6] = fbit(bitf(s[6]) + R.drift);
                    s[7] = fbit(bitf(s[7]) + R.advantage);
                    s[8] = fbit(R.slippage_rm); s[9] = fbit(R.price_adv_rm); s[10] = fbit(R.price_drift_rm);
                    s[11] = fbit(R.vwap_rm); s[12] = fbit(R.trade_duration);
                    d = wsub(s[1], s[2]) <= 0;
                    rew = R.reward / tc.reward_scaling_quo;
                    iw[0] = R.quant_left; iw[1] = d; iw[2] = fbit(R.slippage); iw[3] = fbit(R.vwap_rm);
                    iw[4] = fbit(R.drift); iw[5] = fbit(R.advantage); iw[6] = R.doom_quant; iw[7] = s[3];
                    iw[8] = fbit(R.reward_info);
                }
                if (emit & (l == 0)) {
                    rew_out[(size_t)e * c.n_agents + ag] = rew;
                    dones_out[(size_t)e * c.n_agents + ag] = (u8)(d != 0);
                }
                if (info) {
                    i32 v = 0;
                    for (int k = 0; k < HFTLOB_INFO_AGENT_WORDS; ++k) if (l == k) v = iw[k];
                    if (l < HFTLOB_INFO_AGENT_WORDS) info[HFTLOB_INFO_WORLD_WORDS + ag * HFTLOB_INFO_AGENT_WORDS + l] = v;
                }
                SUBSTAMP(to0);
                if (!all) {  // stepped state + obs survive only when the episode continues
                    i32 v = 0;
                    for (int k = 0; k < 13; ++k) if (l == k) v = s[k];
                    if (l < nw) st[l] = v;
#ifndef HFTLOB_KO_OBS  // timing knockout builds only (wrong results)
                    if (emit)
                        write_obs<false>(c, tc, wv, s, obs_out + ((size_t)e * c.n_agents + ag) * c.obs_stride, d != 0,
                                         ftime);
#endif
                }
                if (obs_raw_out)  // the stepped state's raw obs, also on an episode's last step (info)
                    write_obs<true>(c, tc, wv, s, obs_raw_out + ((size_t)e * c.n_agents + ag) * c.obs_stride, false,
                                    ftime);
                STAMP_ACC(acc_obs, to0);
                st += nw;
            }
        }
    }
    STAMP(t_rewards);
    // ---- (F) world state + info
    const float new_mid = X.last_mid;
    if (info) {
        const float ava = wave_fsum(pa_acc) / (float)M, avb = wave_fsum(pb_acc) / (float)M;
        i32 wv_[HFTLOB_INFO_WORLD_WORDS] = {win, fbit(new_mid), wadd(step, 1), last_t0, last_t1, wsub(oidc, A),
                                            last_p_a, last_p_b, fbit(ava), fbit(avb), fbit(dt), (i32)X.ep_done,
                                            (i32)abort_any, wsub(last_p_a, last_p_b)};
        i32 v = 0;
        for (int k = 0; k < HFTLOB_INFO_WORLD_WORDS; ++k) if (l == k) v = wv_[k];
        if (l < HFTLOB_INFO_WORLD_WORDS) info[l] = v;
    }
    if (emit & (l == 0)) done_all_out[e] = (u8)all;
#ifdef HFTLOB_STAMPS
    if (info && l == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        info[0] = (i32)(t_agents - t_start); info[1] = (i32)(t_book - t_agents);
        info[2] = (i32)(t_rewards - t_book); info[3] = (i32)(t_end - t_rewards); info[4] = (i32)all;
#ifndef HFTLOB_STAMPS_COARSE
        info[5] = (i32)(t_keys - t_start); info[6] = (i32)(t_load - t_keys); info[7] = (i32)(t_rows - t_load);
        info[8] = (i32)(t_agents - t_rows);
#else
        info[5] = info[6] = info[7] = info[8] = 0;
        (void)t_keys; (void)t_load; (void)t_rows;
#endif
        info[9] = (i32)acc_act; info[10] = (i32)acc_cnl; info[11] = (i32)acc_flt;
        info[12] = (i32)acc_mmr; info[13] = (i32)acc_exr; info[14] = (i32)acc_obs;
        info[15] = (i32)(__builtin_amdgcn_s_memrealtime() - rt_start);
    }
#endif
    if (all) {  // auto-reset: MARLEnv.step selects reset(key_reset) for state and obs
        env_reset_dev<S>(c, key_reset, init_states, rec, emit ? obs_out + (size_t)e * c.n_agents * c.obs_stride : nullptr,
                         B.vs, B.vt, ftime);
        return true;
    }
    if (l == 0) {
        rec[c.off_loaded + LD_STEP] = wadd(step, 1);
        i32* W = rec + c.off_world;
        W[W_T0] = last_t0; W[W_T1] = last_t1; W[W_OIDC] = wsub(oidc, A); W[W_MID] = fbit(new_mid); W[W_DT] = fbit(dt);
    }
    return false;
}

// One launch = one batched step.  Env slices: block e steps record e of the
// (offset) buffers, and derives its Speed_test step key as env key_e0 + e of a
// split over key_n envs (split(master, key_n + 1)[key_e0 + e + 1]); a full-batch
// launch has key_e0 = 0, key_n = n_env.  Block 0 writes the carried master key
// split(master, key_n + 1)[0] to master_out.
template <int S, int NFIX, bool RC, bool RA = false>
__global__ __launch_bounds__(64) void k_env_step(hftlob_env_cfg c, int n_env, int key_e0, int key_n,
                                                 const u32* __restrict__ keys, const u32* __restrict__ master,
                                                 u32* __restrict__ master_out, i32* __restrict__ actions_io,
                                                 const i32* __restrict__ msg_data, const i32* __restrict__ init_states,
                                                 i32* __restrict__ state, hftlob_step_out out) {
    one_wave();
    extern __shared__ __attribute__((aligned(16))) i32 lds[];
    const int e = blockIdx.x;
    if (e >= n_env) return;
    Key mk{0u, 0u};
    if (master) mk = Key{master[0], master[1]};
    u32 fl = 0;
    env_step_dev<S, NFIX, RC, RA>(c, key_n, key_e0 + e, e, keys, master != nullptr, mk, actions_io, msg_data, init_states,
                              state, out.obs, out.rewards, out.done_all, out.dones, out.info, out.obs_raw, out.msgs,
                              out.debug, lds, false, false, fl);
    if (master && (e == 0) && (lane_id() == 0)) { master_out[0] = mk.a; master_out[1] = mk.b; }
}

// Speed_test's whole rollout scan in ONE launch (Speed_test.py:186-196): every env
// (one wave) runs its n_steps steps back to back, so no step boundary waits for the
// batch's slowest env (a wave that finishes a step starts its next one at once).
// Each wave carries its own copy of the master-key chain.  The step body is the
// same env_step_dev as k_env_step; per-iteration opaque copies of the config and
// base pointers keep LICM from hoisting the body's invariant loads and addresses
// out of the step loop (they would stay live across it and double the registers):
// the config pointer stays in the constant address space, so its fields are
// still scalar loads, re-issued once per step.  (Never take &c: that copies the
// struct to scratch.)
typedef const __attribute__((address_space(4))) hftlob_env_cfg kcfg_t;

// Issue priority by projected finish.  An env's work over a rollout depends on its data windows
// (their crossings, full sides, cancels; tools/diag_wavetime.py measures a coefficient of variation
// of the per-env time), and the launch ends with its slowest env, while the 16 waves of a CU share
// the CU's scalar unit and each SIMD's issue slots, and each SIMD's arbiter favours its oldest
// wave: without a rule the 4 waves of a SIMD finish in dispatch order, the youngest last
// (profiles/r03_wavetime_unbalanced.json: the live waves fall 4096 -> 3072 -> 2048 -> 1024).
// After every step a wave projects its end (100 MHz reference clock: elapsed / steps done *
// steps left), publishes it in the table slot of its hardware wave slot and ranks itself among
// the live waves of its SIMD (slots whose projection lies ahead of now; a finished wave's last
// projection is its end, in the past): the quarter due last runs at s_setprio 3, the next at 2,
// and so on (the longest-remaining-first rule for a makespan).  Slots are per hardware wave slot, so concurrent launches never share one; the table
// is zero-initialised device memory of the code object (no allocation).  Scheduling only: no
// result depends on it.
#define WAVE_SLOTS (8 * 16 * 16 * 64)  // XCC (8) x SE (8) x SH (2) x CU (16), x 64 wave slots per CU
static __device__ unsigned long long g_wave_eta[WAVE_SLOTS];  // (static: one per translation unit of the split build)
// the CU's row of the table (64 wave slots) and this wave's slot in it (SIMD * 16 + wave id)
DEV unsigned long long* wave_row(u32 hwid, u32 xcc, u32& slot) {
    const u32 cu = ((xcc & 7u) * 16u + ((hwid >> 13) & 7u) * 2u + ((hwid >> 12) & 1u)) * 16u + ((hwid >> 8) & 15u);
    slot = ((hwid >> 4) & 3u) * 16u + (hwid & 15u);
    return g_wave_eta + (size_t)cu * 64u;
}
// The table row is shared only by the waves of one CU, whose L2 (their XCD's) is common: workgroup
// scope (L1-bypassing loads, write-through stores) keeps the step's load at L2 latency; agent scope
// (coherent across XCDs) sent it past the L2 (+0.2 to +0.8 %, profiles/r05_ab_filter_prio.txt)
#ifndef HFTLOB_PRIO_SCOPE
#define HFTLOB_PRIO_SCOPE __HIP_MEMORY_SCOPE_WORKGROUP
#endif
DEV void balance_prio(unsigned long long* row, u32 slot, unsigned long long r0, int done, int left) {
    const int l = lane_id();
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    const float el = (float)(now - r0);
    const unsigned long long eta = now + (unsigned long long)(el * ((float)left / (float)done));
    if (l == 0) __hip_atomic_store(row + slot, eta, __ATOMIC_RELAXED, HFTLOB_PRIO_SCOPE);
    unsigned long long v = __hip_atomic_load(row + l, __ATOMIC_RELAXED, HFTLOB_PRIO_SCOPE);
    v = (u32)l == slot ? eta : v;
    v = ((u32)l >> 4) == (slot >> 4) ? v : 0ull;  // the wave's own SIMD (A/B: +2.6 % over the whole CU)
    const lmask live = bal(v > now);
    const lmask later = live & bal((v > eta) | ((v == eta) & ((u32)l < slot)));
    const int n = __builtin_popcountll(live), rank = __builtin_popcountll(later);
    const int q = n > 0 ? (4 * rank) / n : 0;  // 0: due last
    if (q == 0) __builtin_amdgcn_s_setprio(3);
    else if (q == 1) __builtin_amdgcn_s_setprio(2);
    else if (q == 2) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
// KB: 1 = the config derives its step keys in batches (kb_ok, checked by the launch code), 0 = it
// does not, -1 = decided at run time (the general-size and rows-alias instantiations).  The metric
// kernel is KB = 1: its loop holds no per-step key derivation.
template <int S, int NFIX, bool RC, bool RA = false, int KB = -1>
__global__ __launch_bounds__(64, 4) void k_env_rollout(hftlob_env_cfg c, int n_env, int key_e0, int key_n, int n_steps,
                                                    int per_step, const u32* __restrict__ master,
                                                    u32* __restrict__ master_out, i32* __restrict__ actions_io,
                                                    const i32* __restrict__ msg_data,
                                                    const i32* __restrict__ init_states, i32* __restrict__ state,
                                                    hftlob_step_out out) {
    one_wave();
    extern __shared__ __attribute__((aligned(16))) i32 lds[];
    const int e = blockIdx.x;
    if (e >= n_env) return;
    Key mk{master[0], master[1]};
    // `c` is the first kernel argument: offset 0 of the kernarg segment (constant address space)
    kcfg_t* kp = (kcfg_t*)__builtin_amdgcn_kernarg_segment_ptr();
    // the book stays in LDS from one step to the next (stored to the record only by the last
    // step); an auto-reset rewrites the record, and the step after it loads the book from there.
    // (The 100/100 instantiation only: in the general-size ones the AMDGPU backend moved the
    // lane masks of the resident branch to VGPRs, which s_ff1's SGPR operand cannot take.)
    bool resident = false;
    u32 fl = 0;
#ifndef HFTLOB_NO_BALANCE
    const unsigned long long bal_r0 = __builtin_amdgcn_s_memrealtime();
    const u32 bal_hwid = __builtin_amdgcn_s_getreg(0xF804), bal_xcc = __builtin_amdgcn_s_getreg(0x7814);
    u32 bal_slot;
    unsigned long long* bal_row = wave_row(bal_hwid, bal_xcc, bal_slot);
#endif
#ifdef HFTLOB_WAVETIME
    // diagnostic build only (tools/diag_wavetime.py): the wave's start time and hardware slot,
    // then each step's end time, into the per-step info rows (words 0..9 of row (t, e))
    const unsigned long long wt_start = __builtin_amdgcn_s_memtime(), wt_rstart = __builtin_amdgcn_s_memrealtime();
    const u32 wt_hwid = __builtin_amdgcn_s_getreg(0xF804), wt_xcc = __builtin_amdgcn_s_getreg(0x7814);
#endif
    // the key batches (step_keys_batch) live after the book in LDS
    const bool kbat = KB < 0 ? kb_ok(c) : KB == 1;
    const int kbw = kb_words(c);
    i32* kbuf = lds + lds_map(c, NFIX > 0 ? NFIX : c.lob.n_orders, NFIX > 0 ? NFIX : c.lob.n_trades, RA).kb;
    // one step of the rollout: Q = true for a step whose outputs are not emitted (per_step = 0, not
    // the last step).  The quiet steps run in a loop of their own, then the emitted ones (per_step =
    // 1: all steps; 0: the last one) in a second loop: the quiet copy of the step body holds no
    // observation / reward-value code, and the constants the emitting copy keeps in registers are
    // not live across the quiet loop
    auto step = [&](auto Q, int t) {
        constexpr bool QT = decltype(Q)::value;
        const size_t o = per_step ? (size_t)t * n_env : 0;
        const int tb = t % KB_STEPS;
        kcfg_t* cp = kp;
        i32* st = state;
        const i32* md = msg_data;
        const i32* is = init_states;
        asm volatile("" : "+s"(cp), "+s"(st), "+s"(md), "+s"(is));
        const hftlob_env_cfg& cc = *(const hftlob_env_cfg*)cp;
        STAMP(kb0);
        if (kbat && tb == 0) step_keys_batch<NFIX == 0>(cc, key_n, key_e0 + e, mk, imin_(KB_STEPS, n_steps - t), kbuf);
        STAMP(kb1);
        const bool ox = !QT;  // (the optional outputs: written by the emitted steps only)
#ifdef HFTLOB_STAMPS_QUIET
        // diagnostic build only: the quiet steps' phase stamps go to their per_step info rows
        const bool ox_info = true;
#else
        const bool ox_info = ox;
#endif
        const bool reset = env_step_dev<S, NFIX, RC, RA, QT, KB>(
            cc, key_n, key_e0 + e, e, nullptr, true, mk, actions_io ? actions_io + o * cc.action_words : nullptr, md,
            is, st, out.obs + o * cc.n_agents * cc.obs_stride, out.rewards + o * cc.n_agents, out.done_all + o,
            out.dones + o * cc.n_agents, ox_info && out.info ? out.info + o * cc.info_words : nullptr,
            ox && out.obs_raw ? out.obs_raw + o * cc.n_agents * cc.obs_stride : nullptr,
            ox && out.msgs ? out.msgs + o * cc.n_msgs * 8 : nullptr,
            ox && out.debug ? out.debug + o * (size_t)HFTLOB_DEBUG_WORDS(cc.lob.n_trades) : nullptr, lds,
            NFIX > 0 && resident, NFIX > 0 && t + 1 < n_steps, fl, kbat ? kbuf + tb * kbw : nullptr, !QT);
        resident = uni(!reset) != 0;  // (uniform: the divergence analysis cannot see it through the reset's lane loops)
        STAMP(bp0);
#ifndef HFTLOB_NO_BALANCE
#ifndef HFTLOB_BALANCE_EVERY
#define HFTLOB_BALANCE_EVERY 1
#endif
        if ((t + 1 < n_steps) && ((t % HFTLOB_BALANCE_EVERY) == 0))
            balance_prio(bal_row, bal_slot, bal_r0, t + 1, n_steps - t - 1);
#endif
#ifdef HFTLOB_STAMPS
        // rollout-only phases beside env_step_dev's stamps: the step-key batch (every KB_STEPS-th
        // step) and the issue-priority update, words 16 / 17 of the step's info row
        if (out.info && per_step && lane_id() == 0) {
            i32* irow = out.info + ((size_t)t * n_env + e) * cc.info_words;
            irow[16] = (i32)(kb1 - kb0);
            irow[17] = (i32)(__builtin_amdgcn_s_memtime() - bp0);
        }
#endif
#ifdef HFTLOB_WAVETIME
        if (out.info && per_step) {
            const unsigned long long now = __builtin_amdgcn_s_memtime(), rnow = __builtin_amdgcn_s_memrealtime();
            const i32 w10[10] = {(i32)(u32)now, (i32)(u32)(now >> 32), (i32)wt_hwid, (i32)wt_xcc, (i32)(u32)wt_start,
                                 (i32)(u32)(wt_start >> 32), (i32)(u32)rnow, (i32)(u32)(rnow >> 32),
                                 (i32)(u32)wt_rstart, (i32)(u32)(wt_rstart >> 32)};
            i32 v = 0;
#pragma unroll
            for (int k = 0; k < 10; ++k) v = lane_id() == k ? w10[k] : v;
            if (lane_id() < 10) out.info[((size_t)t * n_env + e) * cc.info_words + lane_id()] = v;
        }
#endif
    };
    int t = 0;
#ifdef HFTLOB_STAMPS_QUIET  // diagnostic build only: per_step = 1 rollouts run the quiet body too (stamps of the bench's path)
    if (true) {
#else
    if (!per_step) {
#endif
#pragma unroll 1
        for (; t + 1 < n_steps; ++t) step(std::integral_constant<bool, true>{}, t);
    }
#pragma unroll 1
    for (; t < n_steps; ++t) step(std::integral_constant<bool, false>{}, t);
#ifndef HFTLOB_NO_BALANCE
    // the wave is done: its slot's entry becomes a past time, so no neighbour counts it as live
    if (lane_id() == 0) __hip_atomic_store(bal_row + bal_slot, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
#endif
    if ((e == 0) && (lane_id() == 0)) { master_out[0] = mk.a; master_out[1] = mk.b; }
}

// ==================================================== K3/K4: PRNG kernels
#if !defined(HFTLOB_INST)  // (non-template kernels: the main translation unit only)
__global__ void k_sample_actions(hftlob_env_cfg c, int n_env, const u32* __restrict__ keys, i32* __restrict__ actions) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_env) return;
    const bool part = c.prng_partitionable;
    const Key k{keys[2 * e], keys[2 * e + 1]};
    i32* out = actions + (size_t)e * c.action_words;
    for (int t = 0; t < c.n_types; ++t) {
        const hftlob_agent_type_cfg& tc = c.types[t];
        const Key sub = split_key(k, c.n_types, t, part);
        const int w = tc.action_width;
        // Discrete(n_actions) or MultiDiscrete([fixed_quant_value] * w) (spaces.py:57-65)
        const i32 hi = action_hi(tc);
        for (int i = 0; i < tc.n_agents; ++i) {
            const Key ka = split_key(sub, tc.n_agents, i, part);
            for (int j = 0; j < w; ++j) *out++ = randint_vec(ka, w, j, 0, hi, part);
        }
    }
}
__global__ void k_split_keys(int n_env, int n, int part, const u32* __restrict__ keys, u32* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_env * n) return;
    const int e = t / n, j = t % n;
    const Key o = split_key(Key{keys[2 * e], keys[2 * e + 1]}, n, j, part != 0);
    out[2 * (size_t)t] = o.a;
    out[2 * (size_t)t + 1] = o.b;
}

#endif  // !HFTLOB_INST

// ============================================ instantiations (parallel build)
// The Makefile compiles this file HFTLOB_NPARTS + 1 times: part k (HFTLOB_INST = k) explicitly
// instantiates its share of the env-step / rollout kernels, the main translation unit (no
// HFTLOB_INST) declares them extern and holds the small kernels and the C ABI.
#define HFTLOB_STEP_ARGS hftlob_env_cfg, int, int, int, const u32*, const u32*, u32*, i32*, const i32*, const i32*, i32*, \
                         hftlob_step_out
#define HFTLOB_ROLL_ARGS hftlob_env_cfg, int, int, int, int, int, const u32*, u32*, i32*, const i32*, const i32*, i32*, \
                         hftlob_step_out
#define HFTLOB_STEP(P, SS, NF, RC) P template __global__ void k_env_step<SS, NF, RC, false>(HFTLOB_STEP_ARGS);
#define HFTLOB_ROLL(P, SS, NF, RC) P template __global__ void k_env_rollout<SS, NF, RC, false>(HFTLOB_ROLL_ARGS);
#define HFTLOB_PART1(P) P template __global__ void k_env_rollout<2, 100, false, false, 1>(HFTLOB_ROLL_ARGS);
#define HFTLOB_PART2(P) HFTLOB_STEP(P, 2, 100, false)
#define HFTLOB_PART3(P) HFTLOB_ROLL(P, 1, 0, false) HFTLOB_STEP(P, 1, 0, false)
#define HFTLOB_PART4(P) HFTLOB_ROLL(P, 2, 0, false) HFTLOB_STEP(P, 2, 0, false)
#define HFTLOB_PART5(P) HFTLOB_ROLL(P, 4, 0, false) HFTLOB_STEP(P, 4, 0, false)
#define HFTLOB_PART6(P) HFTLOB_ROLL(P, 1, 0, true) HFTLOB_STEP(P, 1, 0, true) HFTLOB_ROLL(P, 2, 0, true)
#define HFTLOB_PART7(P) HFTLOB_STEP(P, 2, 0, true) HFTLOB_ROLL(P, 4, 0, true) HFTLOB_STEP(P, 4, 0, true)
#define HFTLOB_PART8(P) P template __global__ void k_env_rollout<2, 100, false, true>(HFTLOB_ROLL_ARGS); \
                        P template __global__ void k_env_step<2, 100, false, true>(HFTLOB_STEP_ARGS);
#define HFTLOB_PART9(P) P template __global__ void k_env_rollout<2, 100, false, false, 0>(HFTLOB_ROLL_ARGS);
#define HFTLOB_NONE
#if defined(HFTLOB_INST)
#if HFTLOB_INST == 1
HFTLOB_PART1(HFTLOB_NONE)
#elif HFTLOB_INST == 2
HFTLOB_PART2(HFTLOB_NONE)
#elif HFTLOB_INST == 3
HFTLOB_PART3(HFTLOB_NONE)
#elif HFTLOB_INST == 4
HFTLOB_PART4(HFTLOB_NONE)
#elif HFTLOB_INST == 5
HFTLOB_PART5(HFTLOB_NONE)
#elif HFTLOB_INST == 6
HFTLOB_PART6(HFTLOB_NONE)
#elif HFTLOB_INST == 7
HFTLOB_PART7(HFTLOB_NONE)
#elif HFTLOB_INST == 8
HFTLOB_PART8(HFTLOB_NONE)
#elif HFTLOB_INST == 9
HFTLOB_PART9(HFTLOB_NONE)
#endif
#else  // the main translation unit
#if !defined(HFTLOB_SINGLE_TU)
HFTLOB_PART1(extern) HFTLOB_PART2(extern) HFTLOB_PART3(extern) HFTLOB_PART4(extern)
HFTLOB_PART5(extern) HFTLOB_PART6(extern) HFTLOB_PART7(extern) HFTLOB_PART8(extern) HFTLOB_PART9(extern)
#endif

// ================================================================ C ABI
static thread_local char g_err[256] = "";
static int fail(int code, const char* msg) {
    snprintf(g_err, sizeof g_err, "%s", msg);
    return code;
}
static int slot_sets(int n) { return n <= 64 ? 1 : (n <= 128 ? 2 : 4); }

extern "C" {

int hftlob_version(void) { return HFTLOB_ABI_VERSION; }
const char* hftlob_last_error(void) { return g_err; }

static int check_lob(const hftlob_lob_cfg* c) {
    if (!c) return fail(HFTLOB_ENULL, "null cfg");
    if (c->cancel_mode < 0 || c->cancel_mode > 3) return fail(HFTLOB_EINVAL, "bad cancel_mode");
    if (c->type_4_interpretation < 0 || c->type_4_interpretation > 2) return fail(HFTLOB_EINVAL, "bad type_4_interpretation");
    if (c->n_orders < 1 || c->n_orders > HFTLOB_MAX_SLOTS || c->n_trades < 1 || c->n_trades > HFTLOB_MAX_SLOTS)
        return fail(HFTLOB_ESHAPE, "n_orders / n_trades out of range");
    // get_init_id_match's id range [init_id - 2 * book_depth, init_id] must be a plain int32 range
    if (c->book_depth < 0 || (long long)c->init_id - 2LL * c->book_depth < INT_MIN)
        return fail(HFTLOB_EINVAL, "book_depth must be >= 0 and init_id - 2 * book_depth must fit in int32");
    return HFTLOB_OK;
}
static int launch_status() {
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(HFTLOB_ELAUNCH, hipGetErrorString(err));
    return HFTLOB_OK;
}

int hftlob_book_process(const hftlob_lob_cfg* cfg, int n_env, int n_msg, const uint32_t* keys, const int32_t* msgs,
                        int32_t* asks, int32_t* bids, int32_t* trades, int32_t* best_asks, int32_t* best_bids,
                        void* stream) {
    int rc = check_lob(cfg);
    if (rc) return rc;
    if (n_env < 0 || n_msg < 0) return fail(HFTLOB_ESHAPE, "negative size");
    if (n_env == 0) return HFTLOB_OK;
    if (!asks || !bids || !trades || (n_msg > 0 && !msgs)) return fail(HFTLOB_ENULL, "null array");
    if ((best_asks == nullptr) != (best_bids == nullptr)) return fail(HFTLOB_ENULL, "best_asks/best_bids: both or none");
    const bool rc_ = cfg->cancel_mode >= 2;
    if (rc_ && !keys) return fail(HFTLOB_ENULL, "keys required for cancel_mode 2/3");
    const int S = slot_sets(cfg->n_orders > cfg->n_trades ? cfg->n_orders : cfg->n_trades);
    hipStream_t st = (hipStream_t)stream;
    dim3 g(n_env), b(ENV_BLOCK);
    const size_t shm = 4 * ((size_t)12 * cfg->n_orders + 8 * cfg->n_trades + 64 * 4);
#define LAUNCH_BOOK(SS, RC) hipLaunchKernelGGL((k_book_process<SS, RC>), g, b, shm, st, *cfg, n_env, n_msg, keys, msgs, \
                                               asks, bids, trades, best_asks, best_bids)
    if (rc_) {
        if (S == 1) LAUNCH_BOOK(1, true);
        else if (S == 2) LAUNCH_BOOK(2, true);
        else LAUNCH_BOOK(4, true);
    } else {
        if (S == 1) LAUNCH_BOOK(1, false);
        else if (S == 2) LAUNCH_BOOK(2, false);
        else LAUNCH_BOOK(4, false);
    }
#undef LAUNCH_BOOK
    return launch_status();
}

static bool has_fixed_prices(const hftlob_env_cfg* c) {
    for (int t = 0; t < c->n_types; ++t)
        if (c->types[t].kind == HFTLOB_AGENT_EXE && c->types[t].action_space == HFTLOB_EXE_ACT_FIXED_PRICES) return true;
    return false;
}
static int check_env(const hftlob_env_cfg* c) {
    if (!c) return fail(HFTLOB_ENULL, "null cfg");
    int rc = check_lob(&c->lob);
    if (rc) return rc;
    if (c->ep_type != 0 && c->ep_type != 1) return fail(HFTLOB_EINVAL, "ep_type must be 0 fixed_steps / 1 fixed_time");
    if (c->lob.prng_partitionable != c->prng_partitionable) return fail(HFTLOB_EINVAL, "lob.prng_partitionable differs");
    if (c->n_types < 1 || c->n_types > HFTLOB_MAX_TYPES || c->n_agents < 1 || c->n_agents > HFTLOB_MAX_AGENTS)
        return fail(HFTLOB_ESHAPE, "agent counts out of range");
    if (c->n_msgs < 1 || c->n_msgs > HFTLOB_MAX_MSGS || c->n_action_msgs > 64 ||
        c->n_action_msgs + c->n_cancel_msgs > MAX_AGENT_ROWS)
        return fail(HFTLOB_ESHAPE, "message counts out of range");
    if (c->n_data_msg < 1 || c->n_data_rows < c->n_data_msg || c->n_windows < 1)
        return fail(HFTLOB_ESHAPE, "data / window sizes out of range");
    if (c->obs_stride > HFTLOB_MAX_OBS) return fail(HFTLOB_ESHAPE, "obs_stride too large");
    if (c->tick_size < 1) return fail(HFTLOB_EINVAL, "tick_size must be >= 1");
    int agents = 0;
    for (int t = 0; t < c->n_types; ++t) {
        const hftlob_agent_type_cfg& tc = c->types[t];
        agents += tc.n_agents;
        if (tc.kind == HFTLOB_AGENT_MM) {
            if (tc.action_space < 0 || tc.action_space > HFTLOB_MM_ACT_SIMPLE) return fail(HFTLOB_EINVAL, "MM action_space");
            if ((tc.action_space == HFTLOB_MM_ACT_BOB_RL || tc.action_space == HFTLOB_MM_ACT_BOB_STRATEGY) &&
                tc.bob_v0 <= 0)
                return fail(HFTLOB_EINVAL, "bob_v0 must be positive");
            if (tc.n_action_msgs != 2 || tc.n_msgs != 4) return fail(HFTLOB_EINVAL, "MM message counts");
            if (tc.action_width != 1) return fail(HFTLOB_EINVAL, "MM action_width must be 1");
            if (tc.observation_space < 0 || tc.observation_space > HFTLOB_MM_OBS_MESSAGES)
                return fail(HFTLOB_EINVAL, "MM observation_space");
        } else if (tc.kind == HFTLOB_AGENT_EXE) {
            const int a = tc.action_space;
            const int na = a == HFTLOB_EXE_ACT_FIXED_QUANTS_COMPLEX ? 4
                         : a == HFTLOB_EXE_ACT_FIXED_QUANTS_1MSG    ? 1
                         : a == HFTLOB_EXE_ACT_FIXED_PRICES         ? tc.n_actions : 2;
            if (a < 0 || a > HFTLOB_EXE_ACT_FIXED_PRICES) return fail(HFTLOB_EINVAL, "EXE action_space");
            if (a == HFTLOB_EXE_ACT_FIXED_PRICES && (tc.n_actions < 1 || tc.n_actions > 4))
                return fail(HFTLOB_EINVAL, "fixed_prices: n_actions must be 1..4 (exec_env.py:1042-1073)");
            if (tc.action_width != (a == HFTLOB_EXE_ACT_FIXED_PRICES ? tc.n_actions : 1))
                return fail(HFTLOB_EINVAL, "EXE action_width");
            if (tc.n_action_msgs != na || tc.n_msgs != 2 * na) return fail(HFTLOB_EINVAL, "EXE message counts");
            if (a == HFTLOB_EXE_ACT_TWAP && c->ep_type != 0) return fail(HFTLOB_EINVAL, "twap needs fixed_steps");
            if (tc.observation_space < 0 || tc.observation_space > HFTLOB_EXE_OBS_SIMPLEST_CASE)
                return fail(HFTLOB_EINVAL, "EXE observation_space");
        } else return fail(HFTLOB_EINVAL, "unknown agent kind");
    }
    if (agents != c->n_agents) return fail(HFTLOB_EINVAL, "n_agents mismatch");
    int words = 0;
    for (int t = 0; t < c->n_types; ++t) words += c->types[t].n_agents * c->types[t].action_width;
    if (words != c->action_words) return fail(HFTLOB_EINVAL, "action_words mismatch");
    return HFTLOB_OK;
}

// the kernels' copy of the config: tick_magic for tick_floordiv (a caller's value is ignored)
static hftlob_env_cfg kernel_cfg(const hftlob_env_cfg* cfg) {
    hftlob_env_cfg c = *cfg;
    const uint32_t d = (uint32_t)c.tick_size;  // >= 1 (check_env)
    const int l = d > 1u ? 32 - __builtin_clz(d - 1u) : 0;
    c.tick_magic = (uint32_t)((((unsigned __int128)1 << (31 + l)) + d - 1u) / d);
    return c;
}

int hftlob_env_reset(const hftlob_env_cfg* cfg, int n_env, const uint32_t* keys, const int32_t* msg_data,
                     const int32_t* init_states, int32_t* state, const hftlob_step_out* out, void* stream) {
    int rc = check_env(cfg);
    if (rc) return rc;
    (void)msg_data;
    if (n_env < 0) return fail(HFTLOB_ESHAPE, "negative n_env");
    if (n_env == 0) return HFTLOB_OK;
    if (!keys || !init_states || !state) return fail(HFTLOB_ENULL, "null array");
    float* obs = out ? out->obs : nullptr;
    const int S = slot_sets(cfg->lob.n_orders > cfg->lob.n_trades ? cfg->lob.n_orders : cfg->lob.n_trades);
    hipStream_t st = (hipStream_t)stream;
    dim3 g(n_env), b(ENV_BLOCK);
    const hftlob_env_cfg kc = kernel_cfg(cfg);
    if (S == 1) hipLaunchKernelGGL(k_env_reset<1>, g, b, 0, st, kc, n_env, keys, init_states, state, obs);
    else if (S == 2) hipLaunchKernelGGL(k_env_reset<2>, g, b, 0, st, kc, n_env, keys, init_states, state, obs);
    else hipLaunchKernelGGL(k_env_reset<4>, g, b, 0, st, kc, n_env, keys, init_states, state, obs);
    return launch_status();
}

// dynamic LDS of one env's workgroup: [agent rows][action extras][book] (see env_step_dev)
#ifndef HFTLOB_LDS_FLOOR
#define HFTLOB_LDS_FLOOR 0
#endif
// the 100/100 kernel (launched for these configs; the others take the general-size kernels)
static bool nfix_kernel(const hftlob_env_cfg* cfg) {
    return cfg->lob.cancel_mode < 2 && cfg->lob.n_orders == 100 && cfg->lob.n_trades == 100 && cfg->ep_type == 0 &&
           !has_fixed_prices(cfg);
}
// the rows-in-trades layout where it raises the envs a CU holds: the 100/100 kernel, rows that
// fit (rows_in_trades) and a per-env LDS above the 16 waves' share of a CU (160 KB / 16)
static bool use_rows_alias(const hftlob_env_cfg* cfg) {
    return nfix_kernel(cfg) && rows_in_trades(*cfg, cfg->lob.n_trades) &&
           4 * lds_map(*cfg, cfg->lob.n_orders, cfg->lob.n_trades, false).words > 160 * 1024 / 16;
}
static size_t env_shm(const hftlob_env_cfg* cfg) {
    const size_t b = 4 * (size_t)lds_map(*cfg, cfg->lob.n_orders, cfg->lob.n_trades, use_rows_alias(cfg)).words;
    return b < (size_t)HFTLOB_LDS_FLOOR ? (size_t)HFTLOB_LDS_FLOOR : b;
}

static int env_step_launch(const hftlob_env_cfg* cfg, int n_env, int key_e0, int key_n, const uint32_t* keys,
                           const uint32_t* key_in, uint32_t* key_out, int32_t* actions, const int32_t* msg_data,
                           const int32_t* init_states, int32_t* state, const hftlob_step_out* out, void* stream) {
    if (!out->obs || !out->rewards || !out->done_all || !out->dones) return fail(HFTLOB_ENULL, "null output");
    const int S = slot_sets(cfg->lob.n_orders > cfg->lob.n_trades ? cfg->lob.n_orders : cfg->lob.n_trades);
    hipStream_t st = (hipStream_t)stream;
    dim3 g(n_env), b(ENV_BLOCK);
    const size_t shm = env_shm(cfg);
    const hftlob_env_cfg kc = kernel_cfg(cfg);
#define LAUNCH_STEP(SS, NF, RC) hipLaunchKernelGGL((k_env_step<SS, NF, RC>), g, b, shm, st, kc, n_env, key_e0, key_n, keys, \
                                               key_in, key_out, actions, msg_data, init_states, state, *out)
    if (cfg->lob.cancel_mode >= 2) {  // random cancel fallback: general sizes only
        if (S == 1) LAUNCH_STEP(1, 0, true);
        else if (S == 2) LAUNCH_STEP(2, 0, true);
        else LAUNCH_STEP(4, 0, true);
    } else if (nfix_kernel(cfg)) {  // the 100/100 kernel has no MultiDiscrete / fixed_prices path
        if (use_rows_alias(cfg)) hipLaunchKernelGGL((k_env_step<2, 100, false, true>), g, b, shm, st, kc, n_env, key_e0,
                                                    key_n, keys, key_in, key_out, actions, msg_data, init_states, state, *out);
        else LAUNCH_STEP(2, 100, false);
    }
    else if (S == 1) LAUNCH_STEP(1, 0, false);
    else if (S == 2) LAUNCH_STEP(2, 0, false);
    else LAUNCH_STEP(4, 0, false);
#undef LAUNCH_STEP
    return launch_status();
}

// all n_steps of a rollout in one k_env_rollout launch (see there)
static int env_rollout_launch(const hftlob_env_cfg* cfg, int n_env, int key_e0, int key_n, int n_steps, int per_step,
                              const uint32_t* key_in, uint32_t* key_out, int32_t* actions, const int32_t* msg_data,
                              const int32_t* init_states, int32_t* state, const hftlob_step_out* out, void* stream) {
    const int S = slot_sets(cfg->lob.n_orders > cfg->lob.n_trades ? cfg->lob.n_orders : cfg->lob.n_trades);
    hipStream_t st = (hipStream_t)stream;
    dim3 g(n_env), b(ENV_BLOCK);
    const size_t shm = env_shm(cfg);
    const hftlob_env_cfg kc = kernel_cfg(cfg);
#define LAUNCH_ROLL(SS, NF, RC) hipLaunchKernelGGL((k_env_rollout<SS, NF, RC>), g, b, shm, st, kc, n_env, key_e0, key_n, \
                                               n_steps, per_step, key_in, key_out, actions, msg_data, init_states, \
                                               state, *out)
    if (cfg->lob.cancel_mode >= 2) {
        if (S == 1) LAUNCH_ROLL(1, 0, true);
        else if (S == 2) LAUNCH_ROLL(2, 0, true);
        else LAUNCH_ROLL(4, 0, true);
    } else if (nfix_kernel(cfg)) {
        if (use_rows_alias(cfg)) hipLaunchKernelGGL((k_env_rollout<2, 100, false, true>), g, b, shm, st, kc, n_env,
                                                    key_e0, key_n, n_steps, per_step, key_in, key_out, actions, msg_data,
                                                    init_states, state, *out);
        else if (kb_ok(*cfg)) hipLaunchKernelGGL((k_env_rollout<2, 100, false, false, 1>), g, b, shm, st, kc, n_env, key_e0,
                                                 key_n, n_steps, per_step, key_in, key_out, actions, msg_data,
                                                 init_states, state, *out);
        else hipLaunchKernelGGL((k_env_rollout<2, 100, false, false, 0>), g, b, shm, st, kc, n_env, key_e0, key_n, n_steps,
                                per_step, key_in, key_out, actions, msg_data, init_states, state, *out);
    }
    else if (S == 1) LAUNCH_ROLL(1, 0, false);
    else if (S == 2) LAUNCH_ROLL(2, 0, false);
    else LAUNCH_ROLL(4, 0, false);
#undef LAUNCH_ROLL
    return launch_status();
}

int hftlob_env_step(const hftlob_env_cfg* cfg, int n_env, const uint32_t* keys, const int32_t* actions,
                    const int32_t* msg_data, const int32_t* init_states, int32_t* state, const hftlob_step_out* out,
                    void* stream) {
    int rc = check_env(cfg);
    if (rc) return rc;
    if (n_env < 0) return fail(HFTLOB_ESHAPE, "negative n_env");
    if (n_env == 0) return HFTLOB_OK;
    if (!keys || !actions || !msg_data || !init_states || !state || !out) return fail(HFTLOB_ENULL, "null array");
    return env_step_launch(cfg, n_env, 0, n_env, keys, nullptr, nullptr, const_cast<int32_t*>(actions), msg_data,
                           init_states, state, out, stream);
}

int hftlob_env_step_sampled(const hftlob_env_cfg* cfg, int n_env, const uint32_t* key_in, uint32_t* key_out,
                            int32_t* actions_out, const int32_t* msg_data, const int32_t* init_states,
                            int32_t* state, const hftlob_step_out* out, void* stream) {
    int rc = check_env(cfg);
    if (rc) return rc;
    if (n_env < 0) return fail(HFTLOB_ESHAPE, "negative n_env");
    if (n_env == 0) return HFTLOB_OK;
    if (!key_in || !key_out || !msg_data || !init_states || !state || !out) return fail(HFTLOB_ENULL, "null array");
    if (key_in == key_out) return fail(HFTLOB_EINVAL, "key_in and key_out must be distinct buffers");
    return env_step_launch(cfg, n_env, 0, n_env, nullptr, key_in, key_out, actions_out, msg_data, init_states, state, out,
                           stream);
}

// Rollout: the batch is cut into G contiguous env slices, each stepped on a
// stream of its own (forked from / joined back to the caller's stream with
// events).  A step's launch waits only for the same slice's previous step, so
// the slow envs at the end of one slice's step overlap the other slices' next
// steps instead of idling the CUs at every step boundary.  Every slice carries
// its own copy of the master key chain in a ping-pong pair of the CALLER's
// key_scratch buffer (so rollouts on different caller streams never share
// device scratch).  The library's slice streams are created per device, on
// first use and only as many as the slices need (GPU_MAX_HW_QUEUES is 4).
#define ROLLOUT_MAX_SLICES 4
struct RolloutCtx {
    int n_streams = 0;               // library streams created so far (slices 1..n_streams)
    bool fork_ready = false;
    hipStream_t s[ROLLOUT_MAX_SLICES];
    hipEvent_t fork, join[ROLLOUT_MAX_SLICES];
};
static RolloutCtx g_rollout[64];
static std::mutex g_rollout_mu;

// Device of the caller's stream (the null stream: the current device); the
// calls below run with that device current and restore the caller's after.
struct DeviceGuard {
    int prev = -1, dev = 0;
    int enter(hipStream_t st) {
        if (hipGetDevice(&prev) != hipSuccess) return fail(HFTLOB_ELAUNCH, "hipGetDevice");
        dev = prev;
        if (st && hipStreamGetDevice(st, &dev) != hipSuccess) return fail(HFTLOB_ELAUNCH, "hipStreamGetDevice");
        if (dev < 0 || dev >= 64) return fail(HFTLOB_ELAUNCH, "device index out of range");
        if (dev != prev && hipSetDevice(dev) != hipSuccess) return fail(HFTLOB_ELAUNCH, "hipSetDevice");
        return HFTLOB_OK;
    }
    ~DeviceGuard() {
        if (prev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
};

// the device's slice streams 1..G-1 and events; created outside any stream capture
// by hftlob_rollout_prepare (or lazily here).  A partial failure destroys what it made.
static int rollout_ctx(int dev, int G, RolloutCtx** out) {
    std::lock_guard<std::mutex> lock(g_rollout_mu);
    RolloutCtx& r = g_rollout[dev];
    if (!r.fork_ready) {
        if (hipEventCreateWithFlags(&r.fork, hipEventDisableTiming) != hipSuccess)
            return fail(HFTLOB_ELAUNCH, "rollout fork event creation");
        r.fork_ready = true;
    }
    while (r.n_streams < G - 1) {
        const int g = r.n_streams + 1;
        if (hipStreamCreateWithFlags(&r.s[g], hipStreamNonBlocking) != hipSuccess)
            return fail(HFTLOB_ELAUNCH, "rollout stream creation");
        if (hipEventCreateWithFlags(&r.join[g], hipEventDisableTiming) != hipSuccess) {
            (void)hipStreamDestroy(r.s[g]);
            return fail(HFTLOB_ELAUNCH, "rollout join event creation");
        }
        r.n_streams = g;
    }
    *out = &r;
    return HFTLOB_OK;
}

int hftlob_env_lds_bytes(const hftlob_env_cfg* cfg) {
    const int rc = check_env(cfg);
    return rc ? rc : (int)env_shm(cfg);
}

int hftlob_env_launch_info(const hftlob_env_cfg* cfg, hftlob_launch_info* out) {
    const int rc = check_env(cfg);
    if (rc) return rc;
    if (!out) return fail(HFTLOB_ENULL, "null out");
    // the selection env_step_launch / env_rollout_launch make
    const bool rcm = cfg->lob.cancel_mode >= 2, nf = !rcm && nfix_kernel(cfg);
    out->slot_sets = nf ? 2 : slot_sets(cfg->lob.n_orders > cfg->lob.n_trades ? cfg->lob.n_orders : cfg->lob.n_trades);
    out->nfix = nf ? 100 : 0;
    out->random_cancel = rcm ? 1 : 0;
    out->rows_alias = nf && use_rows_alias(cfg) ? 1 : 0;
    out->lds_bytes = (int)env_shm(cfg);
    out->tick_magic = kernel_cfg(cfg).tick_magic;
    out->key_batch = kb_ok(*cfg) ? 1 : 0;
    return HFTLOB_OK;
}

int hftlob_rollout_prepare(int n_slices, void* stream) {
    if (n_slices < 0 || n_slices > ROLLOUT_MAX_SLICES) return fail(HFTLOB_EINVAL, "n_slices must be 0..4");
    if (n_slices <= 1) return HFTLOB_OK;  // no library stream needed
    DeviceGuard dg;
    int rc = dg.enter((hipStream_t)stream);
    if (rc) return rc;
    RolloutCtx* R = nullptr;
    return rollout_ctx(dg.dev, n_slices, &R);
}

int hftlob_env_rollout_sampled(const hftlob_env_cfg* cfg, int n_env, int key_e0, int key_n, int n_steps,
                               const uint32_t* key_in, uint32_t* key_out, uint32_t* key_scratch,
                               int32_t* actions_out, const int32_t* msg_data, const int32_t* init_states,
                               int32_t* state, const hftlob_step_out* out, int per_step, int n_slices, void* stream) {
    int rc = check_env(cfg);
    if (rc) return rc;
    if (n_env < 0 || n_steps < 0) return fail(HFTLOB_ESHAPE, "negative n_env / n_steps");
    if (key_e0 < 0 || key_n < key_e0 + n_env) return fail(HFTLOB_ESHAPE, "key_e0 / key_n: need 0 <= key_e0, key_e0 + n_env <= key_n");
    if (n_slices < 0 || n_slices > ROLLOUT_MAX_SLICES) return fail(HFTLOB_EINVAL, "n_slices must be 0..4");
    if (n_env == 0 || n_steps == 0) return HFTLOB_OK;
    if (!key_in || !key_out || (n_slices > 0 && !key_scratch) || !msg_data || !init_states || !state || !out)
        return fail(HFTLOB_ENULL, "null array");
    if (!out->obs || !out->rewards || !out->done_all || !out->dones) return fail(HFTLOB_ENULL, "null output");
    if (key_in == key_out) return fail(HFTLOB_EINVAL, "key_in and key_out must be distinct buffers");
    hipStream_t caller = (hipStream_t)stream;
    DeviceGuard dg;
    if ((rc = dg.enter(caller))) return rc;
    if (n_slices == 0)  // one launch: every env runs its n_steps back to back
        return env_rollout_launch(cfg, n_env, key_e0, key_n, n_steps, per_step, key_in, key_out, actions_out,
                                  msg_data, init_states, state, out, caller);
    const int G = n_slices < n_env ? n_slices : n_env;
    RolloutCtx* R = nullptr;
    if ((rc = rollout_ctx(dg.dev, G, &R))) return rc;
    if (G > 1 && hipEventRecord(R->fork, caller) != hipSuccess) return fail(HFTLOB_ELAUNCH, "fork event");
    const size_t na = (size_t)cfg->n_agents;
    int forked = 1;  // slices whose stream waits on the fork (slice 0 runs on the caller's stream)
    for (int g = 0; g < G && !rc; ++g) {
        const int e0 = (int)((long)n_env * g / G), e1 = (int)((long)n_env * (g + 1) / G), ne = e1 - e0;
        hipStream_t st = g > 0 ? R->s[g] : caller;
        if (g > 0) {
            if (hipStreamWaitEvent(st, R->fork, 0) != hipSuccess) { rc = fail(HFTLOB_ELAUNCH, "fork wait"); break; }
            forked = g + 1;
        }
        uint32_t* kb = key_scratch + 4 * g;  // this slice's ping-pong pair
        for (int t = 0; t < n_steps && !rc; ++t) {
            const size_t o = per_step ? (size_t)t * n_env + e0 : (size_t)e0;
            hftlob_step_out so;
            so.obs = out->obs + o * na * cfg->obs_stride;
            so.rewards = out->rewards + o * na;
            so.done_all = out->done_all + o;
            so.dones = out->dones + o * na;
            so.info = out->info ? out->info + o * cfg->info_words : nullptr;
            so.obs_raw = out->obs_raw ? out->obs_raw + o * na * cfg->obs_stride : nullptr;
            so.msgs = out->msgs ? out->msgs + o * (size_t)cfg->n_msgs * 8 : nullptr;
            so.debug = out->debug ? out->debug + o * (size_t)HFTLOB_DEBUG_WORDS(cfg->lob.n_trades) : nullptr;
            const uint32_t* kin = t == 0 ? key_in : kb + 2 * ((t - 1) & 1);
            uint32_t* kout = t == n_steps - 1 ? (g == 0 ? key_out : kb + 2 * (t & 1)) : kb + 2 * (t & 1);
            int32_t* acts = actions_out ? actions_out + o * cfg->action_words : nullptr;
            rc = env_step_launch(cfg, ne, key_e0 + e0, key_n, nullptr, kin, kout, acts, msg_data, init_states,
                                 state + (size_t)e0 * cfg->rec_words, &so, st);
        }
    }
    // join every forked slice back into the caller's stream, also after a failed launch, so
    // the caller stays ordered after the work already enqueued (and a capture stays joined)
    for (int g = 1; g < forked; ++g) {
        if (hipEventRecord(R->join[g], R->s[g]) != hipSuccess || hipStreamWaitEvent(caller, R->join[g], 0) != hipSuccess)
            if (!rc) rc = fail(HFTLOB_ELAUNCH, "join event");
    }
    return rc;
}

int hftlob_sample_actions(const hftlob_env_cfg* cfg, int n_env, const uint32_t* keys, int32_t* actions, void* stream) {
    if (!cfg) return fail(HFTLOB_ENULL, "null cfg");
    if (cfg->n_types < 1 || cfg->n_types > HFTLOB_MAX_TYPES) return fail(HFTLOB_ESHAPE, "n_types");
    if (n_env < 0) return fail(HFTLOB_ESHAPE, "negative n_env");
    if (n_env == 0) return HFTLOB_OK;
    if (!keys || !actions) return fail(HFTLOB_ENULL, "null array");
    hipLaunchKernelGGL(k_sample_actions, dim3((n_env + 255) / 256), dim3(256), 0, (hipStream_t)stream, *cfg, n_env, keys,
                       actions);
    return launch_status();
}

int hftlob_split_keys(int n_env, int n, int partitionable, const uint32_t* keys, uint32_t* out, void* stream) {
    if (n_env < 0 || n < 1) return fail(HFTLOB_ESHAPE, "bad sizes");
    if (n_env == 0) return HFTLOB_OK;
    if (!keys || !out) return fail(HFTLOB_ENULL, "null array");
    const long total = (long)n_env * n;
    hipLaunchKernelGGL(k_split_keys, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n_env, n,
                       partitionable, keys, out);
    return launch_status();
}

}  // extern "C"
#endif  // the main translation unit
