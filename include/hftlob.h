/*
 * hftlob.h — C ABI of the MI355X-native limit-order-book engine and the
 * multi-agent HFT environment step (libhftlob.so, HIP/gfx950).
 *
 * Every entry point takes plain pointers and sizes.  All array pointers are
 * DEVICE pointers (HBM) unless marked [host]; `stream` is a hipStream_t passed
 * as void* (NULL = the legacy default stream).  Nothing here allocates,
 * synchronises or talks to the host inside step/reset, so a caller may capture
 * these calls in a hipGraph.  Functions return 0 on success and a negative
 * HFTLOB_E* code on an invalid config / shape / null pointer; data conditions
 * never raise (the reference's silent semantics are reproduced:
 * -1 index wrap, book-full eviction, trade-log overwrite, slice clamping).
 *
 * Reference interfaces replaced (paths relative to biiiipy/JaxMARL-HFT):
 *   hftlob_book_process  <- jaxob/JaxOrderBookArrays.py:791-823
 *                           scan_through_entire_array_save_bidask(cfg, key,
 *                           msg_array, (asks,bids,trades), N_steps), vmapped;
 *                           with best_asks/best_bids == NULL it is
 *                           scan_through_entire_array (:736-756).
 *   hftlob_env_reset     <- jaxen/marl_env.py:763-770 MARLEnv.reset ->
 *                           reset_env :129-207 (vmapped over envs).
 *   hftlob_env_step      <- jaxen/marl_env.py:775-804 MARLEnv.step (step_env
 *                           :211-709 + auto-reset select), vmapped over envs.
 *   hftlob_sample_actions<- jaxen/Speed_test.py:166-177 (per-env random actions
 *                           via gymnax Discrete.sample = jax.random.randint).
 *   hftlob_split_keys    <- jax.random.split(key, n) (threefry2x32), batched.
 */
#ifndef HFTLOB_H
#define HFTLOB_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HFTLOB_ABI_VERSION 7

#define HFTLOB_OK            0
#define HFTLOB_EINVAL      (-1)   /* bad config value / unsupported option */
#define HFTLOB_ENULL       (-2)   /* required pointer is NULL */
#define HFTLOB_ESHAPE      (-3)   /* size out of the supported range */
#define HFTLOB_ELAUNCH     (-4)   /* HIP launch error (see hftlob_last_error) */

#define HFTLOB_MAX_TYPES   4      /* agent types per env */
#define HFTLOB_MAX_AGENTS  32     /* agents per env, all types */
#define HFTLOB_MAX_SLOTS   256    /* nOrders and nTrades upper bound */
#define HFTLOB_MAX_MSGS    256    /* messages per step upper bound */
#define HFTLOB_MAX_OBS     16     /* observation width upper bound */
#define HFTLOB_INFO_WORLD_WORDS 14
#define HFTLOB_INFO_AGENT_WORDS 24
#define HFTLOB_L2_LEVELS   10     /* get_L2_state levels of world debug_mode (marl_env.py:646-651) */
#define HFTLOB_DEBUG_WORDS(n_trades) (4 * HFTLOB_L2_LEVELS + 8 * (n_trades))

/* ---- engine configuration: JAXLOB_Configuration (jaxob_config.py:12-30) --- */
typedef struct hftlob_lob_cfg {
    int32_t maxint;                /* 2147483647 */
    int32_t init_id;               /* -2 */
    int32_t book_depth;            /* 10 */
    int32_t cancel_mode;           /* 0 STRICT_BY_ID, 1 INCLUDE_INITS, 2 RANDOM, 3 RANDOM_LARGE */
    int32_t type_4_interpretation; /* 0 IOC, 1 LIM, 2 MKT */
    int32_t check_book_fill;       /* bool */
    int32_t n_orders;              /* slots per book side (nOrders) */
    int32_t n_trades;              /* trade-log rows (nTrades) */
    int32_t prng_partitionable;    /* cancel_mode 2/3 draws: jax_threefry_partitionable (env cfg: equal to
                                      hftlob_env_cfg.prng_partitionable) */
} hftlob_lob_cfg;

/* ---- agent kinds and the option enums (jaxen/mm_env.py, jaxen/exec_env.py) */
enum { HFTLOB_AGENT_MM = 0, HFTLOB_AGENT_EXE = 1 };
enum { HFTLOB_MM_ACT_FIXED_QUANTS = 0, HFTLOB_MM_ACT_DIRECTIONAL = 1, HFTLOB_MM_ACT_BOB_RL = 2,
       HFTLOB_MM_ACT_BOB_STRATEGY = 3, HFTLOB_MM_ACT_AVST = 4, HFTLOB_MM_ACT_SPREAD_SKEW = 5,
       HFTLOB_MM_ACT_SIMPLE = 6 };
enum { HFTLOB_MM_OBS_BASIC = 0, HFTLOB_MM_OBS_ENGINEERED = 1, HFTLOB_MM_OBS_MESSAGES = 2 };
enum { HFTLOB_MM_REW_PORTFOLIO_VALUE = 0, HFTLOB_MM_REW_BUY_SELL_PNL, HFTLOB_MM_REW_COMPLEX,
       HFTLOB_MM_REW_ZERO_INV, HFTLOB_MM_REW_SPOONER, HFTLOB_MM_REW_SPOONER_DAMPED,
       HFTLOB_MM_REW_SPOONER_ASYM_DAMPED, HFTLOB_MM_REW_SPOONER_ASYM_DAMPED2,
       HFTLOB_MM_REW_SPOONER_SCALED, HFTLOB_MM_REW_DELTA_PORTFOLIO_VALUE };
enum { HFTLOB_PRICE_MID = 0, HFTLOB_PRICE_MID_AVG = 1, HFTLOB_PRICE_FAR_TOUCH = 2,
       HFTLOB_PRICE_NEAR_TOUCH = 3 };
enum { HFTLOB_INVPEN_NONE = 0, HFTLOB_INVPEN_LINEAR, HFTLOB_INVPEN_QUADRATIC,
       HFTLOB_INVPEN_THRESHOLD, HFTLOB_INVPEN_EXP4 };
enum { HFTLOB_EXE_ACT_FIXED_QUANTS_COMPLEX = 0, HFTLOB_EXE_ACT_SIMPLEST_CASE = 1, HFTLOB_EXE_ACT_FIXED_QUANTS_1MSG = 2,
       HFTLOB_EXE_ACT_TWAP = 3, HFTLOB_EXE_ACT_FIXED_PRICES = 4 };
enum { HFTLOB_EXE_OBS_ENGINEERED = 0, HFTLOB_EXE_OBS_BASIC = 1, HFTLOB_EXE_OBS_SIMPLEST_CASE = 2 };
enum { HFTLOB_EXE_REW_NORMAL = 0, HFTLOB_EXE_REW_FINISH_FAST = 1, HFTLOB_EXE_REW_SIMPLEST_CASE = 2 };
enum { HFTLOB_TASK_RANDOM = 0, HFTLOB_TASK_BUY = 1, HFTLOB_TASK_SELL = 2 };

/* One agent type (one entry of MultiAgentConfig.dict_of_agents_configs). */
typedef struct hftlob_agent_type_cfg {
    int32_t kind;                  /* HFTLOB_AGENT_* */
    int32_t n_agents;              /* number_of_agents_per_type[t] */
    int32_t trader_id0;            /* first trader id; agent i has trader_id0 - i */
    int32_t n_actions;
    int32_t n_msgs;                /* num_messages_by_agent */
    int32_t n_action_msgs;         /* num_action_messages_by_agent */
    int32_t obs_dim;
    int32_t action_space;          /* HFTLOB_MM_ACT_* / HFTLOB_EXE_ACT_* */
    int32_t observation_space;     /* HFTLOB_MM_OBS_* / HFTLOB_EXE_OBS_* */
    int32_t reward_function;       /* HFTLOB_MM_REW_* / HFTLOB_EXE_REW_* */
    int32_t normalize;
    int32_t time_delay_obs_act;
    int32_t fixed_quant_value;
    /* market maker */
    int32_t tenth_action_market;   /* tenth_action == "MarketOrder" */
    int32_t sell_buy_all_option;   /* must be 0 */
    int32_t fixed_action_setting;
    int32_t fixed_action;
    int32_t auto_liquidate_threshold;
    int32_t unwind_price_penalty;
    int32_t inv_penalty;           /* HFTLOB_INVPEN_* */
    int32_t reference_price;       /* HFTLOB_PRICE_* (MM: mid/mid_avg/far/near; EXE: mid/far) */
    int32_t unwind_price;          /* HFTLOB_PRICE_* (mid/mid_avg/far) */
    int32_t clip_reward;
    int32_t exclude_extreme_spreads;
    int32_t volume_traded_bonus;   /* 0 none, 1 market_share */
    float   auto_liquidate_alpha;
    float   inv_penalty_lambda;
    float   inv_penalty_quadratic_factor;
    float   inv_penalty_threshold;
    float   reward_scaling_quo;
    float   inventoryPnL_eta;
    float   inventoryPnL_gamma;
    float   rebate_bps;
    float   unrealizedPnL_lambda;
    /* execution */
    int32_t task;                  /* HFTLOB_TASK_* */
    int32_t task_size;
    int32_t n_ticks_in_book;
    int32_t doom_price_penalty;
    float   reward_lambda;
    /* constants the reference forms in Python double, then uses as weak f32 */
    float   rebate_factor;         /* rebate_bps / 10_000 */
    float   one_minus_eta;         /* 1 - inventoryPnL_eta */
    /* market-maker action-space parameters (mm_env.py:1123-1809) */
    int32_t bob_v0;                /* bobRL / bobStrategy base quantity */
    int32_t n_ticks_offset;        /* simple */
    int32_t simple_nothing_action; /* simple: 4-entry tables (else 3) */
    int32_t multiplier_type;       /* spread_skew: 0 "tick", 1 "spread" */
    float   spread_multiplier;     /* spread_skew */
    float   skew_multiplier;       /* spread_skew */
    float   avst_var;              /* AvSt avst_var_parameter */
    float   avst_k;                /* AvSt avst_k_parameter */
    float   avst_log_term[8];      /* AvSt: f32 log(1 + gamma_a / k) per action (host, correctly rounded) */
    /* execution: doom_price_penalty * tick_size when the config gives a non-integer penalty
       (a Python float: the far-touch price is then computed in f32, exec_env.py:1544,1569-1573) */
    int32_t doom_penalty_is_float;
    float   doom_penalty_f32;
    /* action words per agent in the actions buffer: 1 for a Discrete space; n_actions (1..4) for
       the EXE fixed_prices MultiDiscrete([fixed_quant_value] * n_actions) space (exec_env.py:2167-2171) */
    int32_t action_width;
} hftlob_agent_type_cfg;

/*
 * Environment configuration (World_EnvironmentConfig + MultiAgentConfig), and
 * the per-env state RECORD layout.  The host (hftlob/layout.py) fills every
 * field including the offsets; kernels read offsets from here.
 *
 * Per-env record, int32 words (floats stored bit-cast), stride rec_words:
 *   [off_asks]   asks  [n_orders][6]   ask_raw_orders
 *   [off_bids]   bids  [n_orders][6]   bid_raw_orders
 *   [off_trades] trades[n_trades][8]
 *   [off_loaded] init_time[2], window_index, max_steps_in_episode,
 *                start_index, step_counter                  (LoadedEnvState)
 *   [off_best_bids] best_bids [M][2]; [off_best_asks] best_asks [M][2]
 *   [off_world]  time[2], order_id_counter, mid_price(f32), delta_time(f32)
 *   [off_agents] per agent, type order: MM 5 words
 *                {posted_distance_bid, posted_distance_ask, inventory,
 *                 total_PnL(f32), cash_balance(f32)}; EXE 13 words
 *                {init_price(f32), task_to_execute, quant_executed,
 *                 is_sell_task, p_vwap, total_revenue, drift_return,
 *                 advantage_return, slippage_rm, price_adv_rm,
 *                 price_drift_rm, vwap_rm, trade_duration (f32)}
 * The init-state table (one row per data window) holds the first
 * init_rec_words words of the same layout (LoadedEnvState).
 */
typedef struct hftlob_env_cfg {
    hftlob_lob_cfg lob;
    int32_t n_data_msg;            /* n_data_msg_per_step (D) */
    int32_t n_msgs;                /* M = D + sum_t n_agents_t * n_msgs_t */
    int32_t n_action_msgs;         /* A = sum_t n_agents_t * n_action_msgs_t */
    int32_t n_cancel_msgs;         /* C = M - D - A */
    int32_t tick_size;
    int32_t ep_type;               /* 0 fixed_steps, 1 fixed_time (data rows past init_time[0] +
                                      episode_time are masked; EXE engineered obs has 15 fields) */
    int32_t episode_time;
    int32_t window_selector;       /* -1 random */
    int32_t n_windows;
    int32_t n_data_rows;           /* rows of the message-data array */
    int32_t placeholder_order_id;
    int32_t artificial_trader_id;
    int32_t artificial_order_id;
    int32_t order_id_counter_start;
    int32_t shuffle_action_messages;
    int32_t prng_partitionable;    /* 1: jax_threefry_partitionable=True (JAX>=0.5) */
    int32_t n_types;
    int32_t n_agents;              /* all types */
    int32_t obs_stride;            /* floats per agent row in the obs buffer */
    int32_t rec_words, init_rec_words;
    int32_t off_asks, off_bids, off_trades, off_loaded;
    int32_t off_best_bids, off_best_asks, off_world, off_agents;
    int32_t info_words;            /* words per env in the optional info buffer */
    int32_t action_words;          /* sum_t n_agents_t * action_width_t: int32 words per env of actions */
    /* set by the library before each env launch (a caller's value is ignored): the multiplier of
       the exact floor division by tick_size, ceil(2^(31+l) / tick_size), l = ceil(log2 tick_size) */
    uint32_t tick_magic;
    hftlob_agent_type_cfg types[HFTLOB_MAX_TYPES];
} hftlob_env_cfg;

/* Outputs of one batched step / reset.  obs/rewards/dones may not be NULL;
 * info, obs_raw and msgs may be NULL (skipped).  Layouts:
 *   obs      f32   [n_env][n_agents][obs_stride]   (agent order = type order)
 *   rewards  f32   [n_env][n_agents]
 *   done_all bool (uint8 0/1) [n_env]              dones["__all__"]
 *   dones    bool (uint8 0/1) [n_env][n_agents]    dones["agents"]
 *   info     32-bit words [n_env][info_words]: world info then one
 *            HFTLOB_INFO_AGENT_WORDS block per agent (ints, or f32 bit-cast;
 *            field map in hftlob/layout.py)
 *   obs_raw  32-bit words [n_env][n_agents][obs_stride] (step only): each agent's
 *            un-normalised observation of the stepped state, the reference's
 *            info["agents"][t]["obs_raw"] under save_raw_observations
 *            (marl_env.py:684-685: get_observation(..., normalize=False,
 *            flatten=False)), fields in sorted-key order, int32 fields as int32 and
 *            float32 fields as f32 bits (key / dtype map in hftlob/layout.py); not
 *            zeroed for done agents and taken before the auto-reset, as info is
 *   msgs     int32 [n_env][n_msgs][8] (step only): the step's combined message
 *            array [cancels; shuffled actions; data] as processed by the book —
 *            the MM "messages" observation (mm_env.py:2820-2821), and
 *            info["world"]["total_msgs"] under world debug_mode
 *   debug    int32 [n_env][HFTLOB_DEBUG_WORDS(n_trades)] (step only): world
 *            debug_mode's info (marl_env.py:645-656) of the stepped state, taken
 *            before the auto-reset as info is: words [0, 40) lob_state =
 *            get_L2_state(asks, bids, 10) (JaxOrderBookArrays.py:1231-1264: 10 rows
 *            [ask_p, ask_q, bid_p, bid_q], unique ask prices ascending with -1 read
 *            as maxint, unique bid prices descending, missing levels maxint /
 *            -maxint, negative volumes 0), then the step's trade log [n_trades][8]
 *            (info["world"]["trades"]) */
typedef struct hftlob_step_out {
    float*   obs;
    float*   rewards;
    uint8_t* done_all;
    uint8_t* dones;
    int32_t* info;
    int32_t* obs_raw;
    int32_t* msgs;
    int32_t* debug;
} hftlob_step_out;

int         hftlob_version(void);
const char* hftlob_last_error(void);

/* Batched order-book message processing (engine operator).
 * Replaces jax.vmap(scan_through_entire_array_save_bidask) —
 * gymnax_exchange/jaxob/JaxOrderBookArrays.py:791-823 — and, with NULL best
 * arrays, jax.vmap(scan_through_entire_array) — :736-756.
 * msgs      [n_env][n_msg][8]      message rows [type,side,q,p,oid,tid,s,ns]
 * asks,bids [n_env][n_orders][6]   in/out
 * trades    [n_env][n_trades][8]   in/out (caller initialises, e.g. all -1)
 * best_asks,best_bids [n_env][n_msg][2] out: (price, qty) after every message,
 *           NULL for both = scan_through_entire_array (no per-message output).
 * keys      uint32 [n_env][2]: the scan's `key` argument; message k draws from
 *           split(key, n_msg)[k] (get_random_id_match, :141-164).  Only read
 *           for cancel_mode 2/3; may be NULL otherwise. */
int hftlob_book_process(const hftlob_lob_cfg* cfg /*[host]*/, int n_env, int n_msg, const uint32_t* keys,
                        const int32_t* msgs, int32_t* asks, int32_t* bids, int32_t* trades,
                        int32_t* best_asks, int32_t* best_bids, void* stream);

/* Batched MARLEnv.reset — replaces jax.vmap(env.reset, (0, None)):
 * gymnax_exchange/jaxen/marl_env.py:763-770 (reset_env :129-207,
 * BaseLOBEnv.reset_env base_env.py:218-234).
 * keys uint32 [n_env][2]; state [n_env][rec_words].
 * msg_data [n_data_rows][8]; init_states [n_windows][init_rec_words]. */
int hftlob_env_reset(const hftlob_env_cfg* cfg /*[host]*/, int n_env, const uint32_t* keys,
                     const int32_t* msg_data, const int32_t* init_states,
                     int32_t* state, const hftlob_step_out* out /*[host] struct*/, void* stream);

/* Batched MARLEnv.step with auto-reset — replaces
 * jax.vmap(env.step, in_axes=(0, 0, 0, None)): marl_env.py:775-804 (step_env
 * :211-709).  keys uint32 [n_env][2]; actions int32 [n_env][action_words]: agent by agent in
 * type order, action_width words each (== [n_env][n_agents] when every space is Discrete). */
int hftlob_env_step(const hftlob_env_cfg* cfg /*[host]*/, int n_env, const uint32_t* keys,
                    const int32_t* actions, const int32_t* msg_data, const int32_t* init_states,
                    int32_t* state, const hftlob_step_out* out /*[host] struct*/, void* stream);

/* One Speed_test rollout step in a single launch — replaces the body of
 * _env_step in gymnax_exchange/jaxen/Speed_test.py:165-185:
 *   rng, *step_keys = split(rng, n_env + 1)      (key_in -> key_out, step keys)
 *   actions = hftlob_sample_actions(step_keys)     (written to actions_out if not NULL)
 *   hftlob_env_step(step_keys, actions, ...)
 * key_in / key_out: uint32 [2] device buffers, distinct (every env reads
 * key_in; key_out receives split(key_in, n_env + 1)[0]). */
int hftlob_env_step_sampled(const hftlob_env_cfg* cfg /*[host]*/, int n_env, const uint32_t* key_in,
                            uint32_t* key_out, int32_t* actions_out, const int32_t* msg_data,
                            const int32_t* init_states, int32_t* state, const hftlob_step_out* out /*[host] struct*/,
                            void* stream);

/* n_steps consecutive Speed_test rollout steps — replaces the whole
 * jax.lax.scan of Speed_test.py:186-196 (`rollout`): the same results, bit for
 * bit, as n_steps hftlob_env_step_sampled calls with key_out fed back as
 * key_in.  Env e of this call takes the step key
 * split(master, key_n + 1)[key_e0 + e + 1]: a call over the whole batch has
 * key_e0 = 0, key_n = n_env; a rank that owns envs [key_e0, key_e0 + n_env)
 * of a NUM_ENVS = key_n batch sharded over GPUs (ippo_rnn_JAXMARL_pmap.py:292-332)
 * passes its offset, so N ranks together replay the single-device rollout.
 * n_slices = 0: ONE kernel launch for all n_steps; every env (one wavefront)
 * runs its steps back to back with its own copy of the master-key chain, so no
 * step boundary waits for the batch's slowest env (for 100/100-slot books the
 * book also stays in LDS between steps; the last step stores it to `state`).
 * n_slices = 1..4: the envs are cut into n_slices contiguous slices, each stepped
 * by one launch per step: slice 0 on `stream`, the others on library-owned HIP
 * streams of the stream's device, forked from / joined back to it with events
 * (no host synchronisation), so one slice's slowest envs overlap the other
 * slices' next steps.
 * key_scratch: uint32 [n_slices][2][2] device scratch owned by the caller (each
 * slice's copy of the master-key chain; may be NULL for n_slices = 0); one buffer
 * per concurrent caller stream.
 * per_step != 0: out->{obs,rewards,done_all,dones,info} and actions_out hold a
 * leading [n_steps] dimension (step t at offset t * their per-step size);
 * per_step == 0: each step overwrites them (the scan discards them).  key_out
 * receives the master key after n_steps splits.  The slice streams are created
 * on first use; call hftlob_rollout_prepare before capturing a rollout in a
 * hipGraph.  If a launch fails, the slices already enqueued are still joined
 * back into `stream` before the error is returned. */
int hftlob_env_rollout_sampled(const hftlob_env_cfg* cfg /*[host]*/, int n_env, int key_e0, int key_n, int n_steps,
                               const uint32_t* key_in, uint32_t* key_out, uint32_t* key_scratch,
                               int32_t* actions_out, const int32_t* msg_data, const int32_t* init_states,
                               int32_t* state, const hftlob_step_out* out /*[host] struct*/, int per_step,
                               int n_slices, void* stream);

/* Creates the library streams / events hftlob_env_rollout_sampled needs for n_slices
 * slices on the device of `stream` (host-only; idempotent). */
int hftlob_rollout_prepare(int n_slices, void* stream);

/* Dynamic LDS bytes of one env's workgroup in hftlob_env_step / hftlob_env_rollout_sampled
 * for this config (agent rows, action extras, book sides, trade log, pad / filter / scratch rows
 * and the rollout's step-key batches), or a negative HFTLOB_E* code for an invalid cfg
 * (host-only, no device call).  Hosts size launch shapes from it (how many envs a CU holds at
 * once); it replaces nothing in the reference, whose XLA compiler sizes its own buffers. */
int hftlob_env_lds_bytes(const hftlob_env_cfg* cfg /*[host]*/);

/* Which kernel instantiation hftlob_env_step / hftlob_env_rollout_sampled launch for this
 * config, and the launch-derived constants they pass it (host-only, no device call).  Tests
 * use it to assert which code path a parity case ran; it replaces nothing in the reference.
 *   slot_sets     register sets per lane (1, 2 or 4: n_orders / n_trades up to 64 / 128 / 256)
 *   nfix          100: the 100/100-slot specialisation; 0: the general-size kernel
 *   random_cancel 1: the cancel_mode 2/3 (get_random_id_match) instantiation
 *   rows_alias    1: the agents' message rows live inside the trade log (the layout that
 *                 raises the envs a CU holds, e.g. Speed_test's [5, 5] agents)
 *   lds_bytes     dynamic LDS per env workgroup (hftlob_env_lds_bytes)
 *   tick_magic    the multiplier of the exact floor division by tick_size the kernels use,
 *                 ceil(2^(31+l) / tick_size), l = ceil(log2 tick_size)
 *   key_batch     1: hftlob_env_rollout_sampled's persistent launch derives the step keys four
 *                 steps at a time (partitionable keys, <= 3 agents, <= 8 action rows) */
typedef struct hftlob_launch_info {
    int32_t slot_sets, nfix, random_cancel, rows_alias, lds_bytes;
    uint32_t tick_magic;
    int32_t key_batch;
} hftlob_launch_info;
int hftlob_env_launch_info(const hftlob_env_cfg* cfg /*[host]*/, hftlob_launch_info* out /*[host]*/);

/* Speed_test action sampling (Speed_test.py:166-177, gymnax Discrete.sample):
 * for env e with step key k_e,
 * sub = split(k_e, n_types); per type t, agent i:
 * actions[e][agent] = randint(split(sub[t], n_agents_t)[i], 0, n_actions_t), or for
 * MultiDiscrete (from_JAXMARL/spaces.py:57-65) the action_width words
 * randint(split(sub[t], n_agents_t)[i], (width,), 0, fixed_quant_value).
 * actions int32 [n_env][action_words]. */
int hftlob_sample_actions(const hftlob_env_cfg* cfg /*[host]*/, int n_env, const uint32_t* keys,
                          int32_t* actions, void* stream);

/* Batched jax.random.split (threefry2x32; partitionable = jax_threefry_partitionable):
 * out[e][j] = split(keys[e], n)[j]; out [n_env][n][2]. */
int hftlob_split_keys(int n_env, int n, int partitionable, const uint32_t* keys,
                      uint32_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HFTLOB_H */
