"""``MARLEnv`` — the multi-agent LOB environment on the HIP path.

Drop-in for ``gymnax_exchange/jaxen/marl_env.py:MARLEnv`` (:45-804): same
constructor arguments, ``default_params``, ``reset(key, params) -> (obs_list,
state)``, ``step(key, state, actions, params) -> (obs_list, state,
reward_list, dones, info)``, ``action_spaces`` / ``observation_spaces``,
``num_msgs_per_step``.  The reference is written per-env and vmapped by its
callers (``jax.vmap(env.step, in_axes=(0,0,0,None))``); here the env batch
is explicit: ``key`` is uint32 ``[E, 2]``, every state leaf / action / output
carries a leading ``E``.  One ``step`` is ONE kernel launch
(``hftlob_env_step``) over all envs, auto-reset included.

State lives in one int32 tensor ``[E, rec_words]`` (see ``layout.py``);
``MultiAgentState.world_state`` / ``.agent_states`` expose the reference's
pytree field names as zero-copy views.  ``step`` updates the state in place
and returns the same object (callers that rebind ``state = step(...)[1]``, as
every reference caller does, see no difference).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib
from .config import Execution_EnvironmentConfig, MarketMaking_EnvironmentConfig, MultiAgentConfig
from .data.synthetic import LobsterDay, generate_day
from .data.windows import Windows, init_messages, loaded_rows, make_windows
from .engine import book_process_
from .layout import (AGENT_MM, EXE_FLOAT, action_width, EXE_WORDS, INFO_AGENT_WORDS, INFO_EXE, INFO_MM, INFO_WORLD,
                     INFO_WORLD_WORDS, L2_LEVELS, MM_FLOAT, MM_WORDS, EnvLayout, StepOut, debug_words, obs_fields,
                     pack_env_cfg, trader_ids)


# ------------------------------------------------------------------ spaces
class Discrete:
    def __init__(self, n: int):
        self.n, self.shape, self.dtype = int(n), (), torch.int32


class MultiDiscrete:
    """from_JAXMARL/spaces.py:45-70: one categorical per dimension."""
    def __init__(self, num_categories):
        self.n = [int(x) for x in num_categories]
        self.shape, self.dtype = (len(self.n),), torch.int32


class Box:
    def __init__(self, low, high, shape, dtype=torch.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype


# ------------------------------------------------------------------ params
@dataclass
class LoadedEnvParams:               # StatesandParams.py:96-101
    message_data: torch.Tensor       # (N, 8) int32
    book_data: torch.Tensor          # (W, 40) int32
    init_states_array: torch.Tensor  # (W, init_rec_words) int32


@dataclass
class MMEnvParams:                   # StatesandParams.py:111-116
    trader_id: torch.Tensor
    time_delay_obs_act: torch.Tensor
    normalize: torch.Tensor


@dataclass
class ExecEnvParams:                 # StatesandParams.py:119-124
    trader_id: torch.Tensor
    task_size: torch.Tensor
    reward_lambda: torch.Tensor
    time_delay_obs_act: torch.Tensor
    normalize: torch.Tensor


@dataclass
class MultiAgentParams:              # StatesandParams.py:104-108
    loaded_params: LoadedEnvParams
    agent_params: list


# ------------------------------------------------------------------- state
def _iview(buf, off, shape):
    n = int(np.prod(shape)) if shape else 1
    v = buf[:, off:off + n]
    return v.reshape(buf.shape[0], *shape) if shape else v[:, 0]


class WorldState:
    """Views of the world part of the record (WorldState, StatesandParams.py:29-38)."""

    def __init__(self, buf: torch.Tensor, L: EnvLayout):
        self._buf, self._L = buf, L

    def __getattr__(self, name):
        b, L = self.__dict__["_buf"], self.__dict__["_L"]
        nO, nT, M = L.n_orders, L.n_trades, L.n_msgs
        lo, w = L.off_loaded, L.off_world
        table = {
            "ask_raw_orders": lambda: _iview(b, L.off_asks, (nO, 6)),
            "bid_raw_orders": lambda: _iview(b, L.off_bids, (nO, 6)),
            "trades": lambda: _iview(b, L.off_trades, (nT, 8)),
            "init_time": lambda: b[:, lo:lo + 2],
            "window_index": lambda: b[:, lo + 2],
            "max_steps_in_episode": lambda: b[:, lo + 3],
            "start_index": lambda: b[:, lo + 4],
            "step_counter": lambda: b[:, lo + 5],
            "best_bids": lambda: _iview(b, L.off_best_bids, (M, 2)),
            "best_asks": lambda: _iview(b, L.off_best_asks, (M, 2)),
            "time": lambda: b[:, w:w + 2],
            "order_id_counter": lambda: b[:, w + 2],
            "mid_price": lambda: b[:, w + 3:w + 4].view(torch.float32)[:, 0],
            "delta_time": lambda: b[:, w + 4:w + 5].view(torch.float32)[:, 0],
        }
        if name not in table:
            raise AttributeError(name)
        return table[name]()


class AgentStates:
    """Per-type agent state views [E, n_agents] (MMEnvState / ExecEnvState)."""

    def __init__(self, buf, offsets: List[int], kind: int):
        self._buf, self._offs, self._kind = buf, offsets, kind
        self._names = MM_WORDS if kind == AGENT_MM else EXE_WORDS

    def __getattr__(self, name):
        d = self.__dict__
        if name not in d["_names"]:
            raise AttributeError(name)
        k = d["_names"].index(name)
        offs, W = d["_offs"], (5 if d["_kind"] == AGENT_MM else 13)
        o0 = offs[0] + k
        v = d["_buf"][:, o0:o0 + W * (len(offs) - 1) + 1:W]
        return v.view(torch.float32) if name in (MM_FLOAT if d["_kind"] == AGENT_MM else EXE_FLOAT) else v


@dataclass
class MultiAgentState:               # StatesandParams.py:43-47
    buf: torch.Tensor                # (E, rec_words) int32 record
    world_state: WorldState
    agent_states: list

    def clone(self, env: "MARLEnv") -> "MultiAgentState":
        return env._wrap(self.buf.clone())


# -------------------------------------------------------------------- env
class MARLEnv:
    def __init__(self, key, multi_agent_config: MultiAgentConfig, data=None,
                 device=None, prng_partitionable: bool = True, return_info: bool = True,
                 persistent_outputs: bool = False):
        """data: a synthetic ``LobsterDay`` (None = the seeded default day), a ``LoadedDay`` from
        ``hftlob.data.lobster``, or ``"lobster"`` to load ``world_config.dataPath`` /
        ``stock`` / ``timePeriod`` through ``LoadLOBSTER_resample`` as the reference's
        ``BaseLOBEnv.__init__`` does (base_env.py:157-176)."""
        self.multi_agent_config = cfg = multi_agent_config
        self.device = torch.device(device or "cuda")
        w = cfg.world_config
        self.num_agents = sum(cfg.number_of_agents_per_type)
        self.list_of_agents_configs = list(cfg.dict_of_agents_configs.values())
        self.type_names = [a.short_name for a in self.list_of_agents_configs]
        if data is None:
            data = generate_day(seed=20260403, snap_every=w.n_data_msg_per_step * w.start_resolution)
        elif isinstance(data, str):
            if data != "lobster":
                raise ValueError(f"data={data!r}: pass a LobsterDay, a LoadedDay or 'lobster'")
            from .data.lobster import load_from_config
            data = load_from_config(w)
        self.data = data
        self.windows: Windows = make_windows(data, w)
        self.n_windows = len(self.windows.starts)
        self.prng_partitionable = prng_partitionable
        self.cfg_c, self.layout = pack_env_cfg(cfg, self.n_windows, data.msgs.shape[0], prng_partitionable)
        L = self.layout
        self.num_msgs_per_step = L.n_msgs
        self.num_action_msgs_per_step_by_all_agents = L.n_action_msgs
        # exec_env.py:2164-2183 / mm_env.py action_space(): Discrete, or MultiDiscrete for EXE fixed_prices
        self.action_widths = [action_width(a) for a in self.list_of_agents_configs]
        self.action_spaces = [MultiDiscrete([a.fixed_quant_value] * a.n_actions)
                              if isinstance(a, Execution_EnvironmentConfig) and a.action_space == "fixed_prices"
                              else Discrete(a.n_actions) for a in self.list_of_agents_configs]
        self.action_words = int(self.cfg_c.action_words)   # int32 words per env of the actions buffer
        # MM "messages" (mm_env.py:2820-2821): the observation is the step's combined int32 message
        # array [M, 8] (the kernel's msgs output), not a float row
        self.message_obs_types = [isinstance(a, MarketMaking_EnvironmentConfig) and a.observation_space == "messages"
                                  for a in self.list_of_agents_configs]
        self.observation_spaces = [
            Box(-int(w.maxint), int(w.maxint), (a.num_messages_by_agent + w.n_data_msg_per_step, 8), torch.int32)
            if m else  # mm_env.py:3202-3204 declares num_messages_by_agent + D rows
            Box(-1000 if isinstance(a, MarketMaking_EnvironmentConfig) else -10000,
                1000 if isinstance(a, MarketMaking_EnvironmentConfig) else 10000, (d,))
            for a, d, m in zip(self.list_of_agents_configs, L.obs_dims, self.message_obs_types)]
        # info["agents"][t]["obs_raw"] (marl_env.py:684-685): (field, dtype) per type, None = messages
        self.save_raw_observations = bool(w.save_raw_observations)
        self.obs_raw_fields = [obs_fields(a, w) for a in self.list_of_agents_configs]
        # world debug_mode (marl_env.py:645-656): info["world"] also carries the step's trades, its
        # combined messages and the 10-level lob_state of the stepped books
        self.debug_mode = bool(w.debug_mode)
        self.return_info = return_info
        self.persistent_outputs = persistent_outputs
        self._out = None
        self._init_states = self._precompute_init_states()
        # the device every launch goes to: the one this env's tensors were allocated on, fixed here
        # (not whichever device is current at the first launch)
        self._dev_idx = self._init_states.device.index

    # BaseLOBEnv._init_states (base_env.py:298-333) on the GPU engine
    def _precompute_init_states(self) -> torch.Tensor:
        w, L = self.multi_agent_config.world_config, self.layout
        W, dev = self.n_windows, self.device
        first_times = self.data.msgs[self.windows.starts, 6:8].astype(np.int32)
        im = torch.from_numpy(init_messages(self.windows.books, first_times, w.book_depth, w.init_id)).to(dev)
        asks = torch.full((W, w.nOrders, 6), -1, dtype=torch.int32, device=dev)
        bids = torch.full_like(asks, -1)
        trades = torch.full((W, w.nTrades, 8), -1, dtype=torch.int32, device=dev)
        # the init orders are limit adds only, so the scan key (cancel_mode 2/3) is never drawn from
        keys = torch.zeros((W, 2), dtype=torch.int32, device=dev)
        book_process_(w, im.contiguous(), asks, bids, trades, keys=keys, prng_partitionable=self.prng_partitionable)
        rows = loaded_rows(asks.cpu().numpy(), bids.cpu().numpy(), trades.cpu().numpy(), first_times,
                           self.windows, w.n_data_msg_per_step, L.init_rec_words, w)
        return torch.from_numpy(rows).to(dev)

    @property
    def default_params(self) -> MultiAgentParams:
        w = self.multi_agent_config.world_config
        loaded = LoadedEnvParams(message_data=torch.from_numpy(self.data.msgs).to(self.device).contiguous(),
                                 book_data=torch.from_numpy(self.windows.books).to(self.device),
                                 init_states_array=self._init_states)
        plist = []
        for a, ids in zip(self.list_of_agents_configs, trader_ids(self.multi_agent_config)):
            n = len(ids)
            tid = torch.tensor(ids, dtype=torch.int32)
            if isinstance(a, MarketMaking_EnvironmentConfig):
                plist.append(MMEnvParams(tid, torch.full((n,), a.time_delay_obs_act), torch.full((n,), a.normalize)))
            else:
                plist.append(ExecEnvParams(tid, torch.full((n,), a.task_size), torch.full((n,), a.reward_lambda),
                                           torch.full((n,), a.time_delay_obs_act), torch.full((n,), a.normalize)))
        return MultiAgentParams(loaded_params=loaded, agent_params=plist)

    def action_space(self):
        return self.action_spaces

    def observation_space(self):
        return self.observation_spaces

    # -------------------------------------------------------------- plumbing
    def _wrap(self, buf: torch.Tensor) -> MultiAgentState:
        L = self.layout
        agents, a = [], 0
        for t, n in enumerate(self.multi_agent_config.number_of_agents_per_type):
            agents.append(AgentStates(buf, L.agent_offsets[a:a + n], L.agent_kinds[a]))
            a += n
        return MultiAgentState(buf=buf, world_state=WorldState(buf, L), agent_states=agents)

    def _outputs(self, E: int):
        if self.persistent_outputs and self._out is not None and self._out["obs"].shape[0] == E:
            return self._out
        o = self._alloc((E,))
        if self.persistent_outputs:
            self._out = o
        return o

    def _alloc(self, lead: tuple):
        """Output buffers of `lead` (E,) or (T, E) env steps and their hftlob_step_out."""
        L, dev, A = self.layout, self.device, self.num_agents
        want_raw = self.save_raw_observations and self.return_info
        want_dbg = self.debug_mode and self.return_info
        o = {"obs": torch.empty(lead + (A, L.obs_stride), dtype=torch.float32, device=dev),
             "rewards": torch.empty(lead + (A,), dtype=torch.float32, device=dev),
             "done_all": torch.empty(lead, dtype=torch.bool, device=dev),
             "dones": torch.empty(lead + (A,), dtype=torch.bool, device=dev),
             "info": torch.empty(lead + (L.info_words,), dtype=torch.int32, device=dev) if self.return_info else None,
             "obs_raw": torch.empty(lead + (A, L.obs_stride), dtype=torch.int32, device=dev) if want_raw else None,
             "msgs": torch.empty(lead + (L.n_msgs, 8), dtype=torch.int32, device=dev)
             if any(self.message_obs_types) or want_dbg else None,
             "debug": torch.empty(lead + (debug_words(L.n_trades),), dtype=torch.int32, device=dev)
             if want_dbg else None}
        opt = lambda k: _lib.ptr(o[k]) if o[k] is not None else None  # noqa: E731
        o["struct"] = StepOut(_lib.ptr(o["obs"]), _lib.ptr(o["rewards"]), _lib.ptr(o["done_all"]),
                              _lib.ptr(o["dones"]), opt("info"), opt("obs_raw"), opt("msgs"), opt("debug"))
        return o

    def _split_types(self, x: torch.Tensor, obs: bool):
        out, a = [], 0
        for n, d in zip(self.multi_agent_config.number_of_agents_per_type, self.layout.obs_dims):
            out.append(x[:, a:a + n, :d] if obs else x[:, a:a + n])
            a += n
        return out

    def _keys(self, key: torch.Tensor) -> torch.Tensor:
        if key.dtype not in (torch.int32, torch.uint32) or key.dim() != 2 or key.shape[1] != 2:
            raise ValueError("key must be a uint32/int32 tensor [E, 2] (one threefry key per env)")
        return key.to(self.device).contiguous()

    def _actions(self, actions, E: int) -> torch.Tensor:
        """Per-type actions ([E, n_t] Discrete, [E, n_t, width] MultiDiscrete) or one
        [E, action_words] tensor -> the flat int32 actions buffer of the C ABI."""
        if isinstance(actions, torch.Tensor):
            a = actions
        else:
            cols = []
            for x, n, wd in zip(actions, self.multi_agent_config.number_of_agents_per_type, self.action_widths):
                x = torch.as_tensor(x, device=self.device)
                cols.append(x.reshape(E, n * wd))
            a = torch.cat(cols, dim=1)
        return a.to(device=self.device, dtype=torch.int32).reshape(E, self.action_words).contiguous()

    def split_actions(self, flat: torch.Tensor):
        """[E, action_words] -> per-type list ([E, n_t] or [E, n_t, width]), the inverse of _actions."""
        out, k = [], 0
        for n, wd in zip(self.multi_agent_config.number_of_agents_per_type, self.action_widths):
            x = flat[:, k:k + n * wd]
            out.append(x if isinstance(self.action_spaces[len(out)], Discrete) else x.reshape(-1, n, wd))
            k += n * wd
        return out

    def _info_index(self, a: int, n_t: int, k: int) -> torch.Tensor:
        """device index of info word k for agents a..a+n_t-1, cached: no host copy per step
        (so the info dict can be built inside a HIP graph capture)"""
        cache = self.__dict__.setdefault("_info_idx", {})
        key = (a, n_t, k)
        if key not in cache:
            cache[key] = torch.tensor([INFO_WORLD_WORDS + (a + i) * INFO_AGENT_WORDS + k for i in range(n_t)],
                                      dtype=torch.long, device=self.device)
        return cache[key]

    def _info(self, o, E):
        if o["info"] is None:
            return {}
        info = o["info"]
        f = info.view(torch.float32)

        def col(k, isf):
            return f[:, k] if isf else info[:, k]

        world = {n: col(k, isf) for k, (n, isf) in enumerate(INFO_WORLD)}
        world["time"] = torch.stack([world.pop("time_s"), world.pop("time_ns")], 1)
        world["current_step"] = world["step_counter"]
        if o.get("debug") is not None:  # marl_env.py:645-656 (the stepped state's, as the rest of info)
            n4 = 4 * L2_LEVELS
            world["trades"] = o["debug"][:, n4:].reshape(E, self.layout.n_trades, 8)
            world["total_msgs"] = o["msgs"]
            world["lob_state"] = o["debug"][:, :n4]
        agents, a = [], 0
        for n_t in self.multi_agent_config.number_of_agents_per_type:
            fields = INFO_MM if self.layout.agent_kinds[a] == AGENT_MM else INFO_EXE
            d = {}
            for k, (n, isf) in enumerate(fields):
                d[n] = (f if isf else info).index_select(1, self._info_index(a, n_t, k))
            if o.get("obs_raw") is not None:
                d["obs_raw"] = self._obs_raw(o, len(agents), a, n_t, E)
            agents.append(d)
            a += n_t
        return {"world": world, "agents": agents}

    def _obs_raw(self, o, t: int, a: int, n_t: int, E: int):
        """get_observation(normalize=False, flatten=False) of type t's agents: {field: [E, n_t]}
        (int32 / float32 as the reference's dict), or the [E, n_t, M, 8] messages."""
        fields = self.obs_raw_fields[t]
        if fields is None:
            return o["msgs"][:, None].expand(E, n_t, self.layout.n_msgs, 8)
        raw = o["obs_raw"][:, a:a + n_t]
        rawf = raw.view(torch.float32)
        return {n: (rawf if dt == "f" else raw)[:, :, k] for k, (n, dt) in enumerate(fields)}

    def _message_obs(self, o, x: torch.Tensor, t: int, a: int, n_t: int, E: int) -> torch.Tensor:
        """Type t's obs for the MM "messages" space: the combined messages of the step for every
        agent, zeroed where the agent is done but the env is not (marl_env.py:687-698) and where
        the env auto-resets (the reset observation is a blank [M, 8] array)."""
        if not self.message_obs_types[t]:
            return x
        m = o["msgs"][:, None].expand(E, n_t, self.layout.n_msgs, 8)
        zero = o["dones"][:, a:a + n_t] | o["done_all"][:, None]
        return torch.where(zero[:, :, None, None], torch.zeros((), dtype=m.dtype, device=m.device), m)

    def _abi(self, fn: str, *args):
        """Call libhftlob `fn` with this env's device current and torch's current stream OF THAT
        DEVICE appended (the kernels, and the rollout's slice streams, follow the stream).  The
        device context is entered only when another device is current (it costs host time
        before every launch, and the bench's timed region starts before the launch)."""
        f = getattr(_lib.lib(), fn)
        dev = self._dev_index
        if torch.cuda.current_device() == dev:
            rc = f(*args, torch.cuda.current_stream(dev).cuda_stream)
        else:
            with torch.cuda.device(dev):
                rc = f(*args, torch.cuda.current_stream(dev).cuda_stream)
        if rc:
            _lib.check(rc)

    @property
    def _dev_index(self) -> int:
        i = self.__dict__.get("_dev_idx")
        if i is None:
            raise RuntimeError(f"MARLEnv on {self._init_states.device}: the hftlob kernels need a HIP device")
        return i

    # ------------------------------------------------------------------ API
    def reset(self, key: torch.Tensor, params: Optional[MultiAgentParams] = None):
        """MARLEnv.reset / reset_env (marl_env.py:129-207, 763-770) for E envs."""
        if params is None:
            raise ValueError("Params must be provided to reset the environment.")
        keys = self._keys(key)
        E = keys.shape[0]
        buf = torch.empty((E, self.layout.rec_words), dtype=torch.int32, device=self.device)
        o = self._outputs(E)
        self._abi("hftlob_env_reset", C.byref(self.cfg_c), E, _lib.ptr(keys),
                  _lib.ptr(params.loaded_params.message_data), _lib.ptr(params.loaded_params.init_states_array),
                  _lib.ptr(buf), C.byref(o["struct"]))
        obs = self._split_types(o["obs"], True)
        for t, n_t in enumerate(self.multi_agent_config.number_of_agents_per_type):
            if self.message_obs_types[t]:
                # blank messages (mm_env.py:443; the reference's "messages" reset returns None, which its
                # own auto-reset tree_map cannot select against: a blank array keeps step() defined)
                obs[t] = torch.zeros((E, n_t, self.layout.n_msgs, 8), dtype=torch.int32, device=self.device)
        return obs, self._wrap(buf)

    reset_env = reset

    def step(self, key: torch.Tensor, state: MultiAgentState, actions, params: MultiAgentParams,
             reset_state=None):
        """MARLEnv.step (marl_env.py:775-804) for E envs: step_env + auto-reset, one launch."""
        if reset_state is not None:
            raise NotImplementedError("Get obs on the MARL level is not implemented yet")  # as the reference
        keys = self._keys(key)
        E = keys.shape[0]
        acts = self._actions(actions, E)
        o = self._outputs(E)
        self._abi("hftlob_env_step", C.byref(self.cfg_c), E, _lib.ptr(keys), _lib.ptr(acts),
                  _lib.ptr(params.loaded_params.message_data), _lib.ptr(params.loaded_params.init_states_array),
                  _lib.ptr(state.buf), C.byref(o["struct"]))
        return self._results(o, state, E)

    def step_sampled(self, key_in: torch.Tensor, key_out: torch.Tensor, state: MultiAgentState,
                     params: MultiAgentParams, actions_out: Optional[torch.Tensor] = None):
        """One Speed_test rollout step (Speed_test.py:165-185) in one launch:
        ``key_out, *step_keys = split(key_in, E + 1)``, per-type randint actions
        from the step keys (written to ``actions_out`` [E, action_words] if given),
        then ``step``.  key_in / key_out: distinct uint32 [2] device tensors."""
        E = state.buf.shape[0]
        o = self._outputs(E)
        if actions_out is not None and (tuple(actions_out.shape) != (E, self.action_words)
                                        or actions_out.dtype != torch.int32):
            raise ValueError("actions_out must be int32 [E, action_words]")
        self._abi("hftlob_env_step_sampled", C.byref(self.cfg_c), E, _lib.ptr(key_in), _lib.ptr(key_out),
                  _lib.ptr(actions_out), _lib.ptr(params.loaded_params.message_data),
                  _lib.ptr(params.loaded_params.init_states_array), _lib.ptr(state.buf), C.byref(o["struct"]))
        return self._results(o, state, E)

    LDS_PER_CU = 160 * 1024      # MI355X (gfx950) LDS per CU
    ROLLOUT_WAVES_PER_CU = 16    # k_env_rollout: launch_bounds(64, 4), 128 VGPRs -> 4 waves per SIMD
    TUNED_ARCH = "gfx950"        # the device the launch-shape rule below was measured on

    def lds_bytes_per_env(self) -> int:
        """Dynamic LDS of one env's workgroup, from the library (hftlob_env_lds_bytes: env_shm in
        hftlob.hip, the figure its launches use): agent rows, action extras, the two book sides,
        the trade log, the pad / filter / scratch rows and the rollout's key batches."""
        n = int(_lib.lib().hftlob_env_lds_bytes(C.byref(self.cfg_c)))
        if n <= 0:
            _lib.check(n)
        return n

    def launch_info(self) -> dict:
        """The kernel instantiation step / rollout_sampled launch for this config
        (hftlob_env_launch_info): slot_sets, nfix (100 = the 100/100 specialisation),
        random_cancel, rows_alias (agent rows inside the trade log), lds_bytes, tick_magic."""
        info = _lib.LaunchInfo()
        _lib.check(_lib.lib().hftlob_env_launch_info(C.byref(self.cfg_c), C.byref(info)))
        return {k: int(getattr(info, k)) for k, _ in info._fields_}

    def _tuned_device(self) -> bool:
        if not torch.cuda.is_available():
            return True
        return torch.cuda.get_device_properties(self.device).gcnArchName.split(":")[0] == self.TUNED_ARCH

    def resident_envs(self) -> int:
        """Envs of this config the GPU holds at once (workgroups per CU by LDS and by waves; the
        MI355X figures above)."""
        per_cu = min(self.ROLLOUT_WAVES_PER_CU, self.LDS_PER_CU // self.lds_bytes_per_env())
        n_cu = torch.cuda.get_device_properties(self.device).multi_processor_count \
            if torch.cuda.is_available() else 256
        return per_cu * n_cu

    def default_slices(self, n_env: int) -> int:
        """Launch shape of rollout_sampled, measured on 1x MI355X (DESIGN.md section 4,
        tools/sweep_envs.sh, tools/gpu_sweep.sh; profiles/r03_launch_shape_sweep.txt): 0 = one
        persistent launch (every env's steps back to back, its book kept in LDS, issue priority by
        projected finish) whenever its waves of workgroups are full: the whole batch resident, or
        whole multiples of what the GPU holds at once (the metric config, 16 envs per CU:
        512 / 2048 / 4096 / 8192 / 16384 envs at 10.2 / 37.4 / 62.3 / 64.0 / 64.7 M env-steps/s
        against 7.7 / 28.6 / 47.8 / 59.7 / 61.6 M for 2 slices); 2 env slices on their own streams
        when the last wave would be partly empty, as its envs would run whole rollouts after the
        others finish (Speed_test's [5,5] / [10,10] agents at 4000 envs, whose agent rows leave
        room for 14 / 11 envs per CU: 25.1 / 15.7 M against 19.7 / 12.3 M).  On a device other
        than the one this was measured on, 2 slices (they never wait for whole rollouts)."""
        if not self._tuned_device():  # LDS / wave limits of another device are not known here
            return 2
        cap = self.resident_envs()
        if n_env <= cap:
            return 0
        waves = -(-n_env // cap)
        return 0 if n_env >= 0.9 * waves * cap else 2

    def prepare_rollout(self, n_slices: int) -> None:
        """Create the library's slice streams for `n_slices` on this env's device (host-only).
        rollout_sampled does it on first use; call this before capturing a rollout in a HIP graph."""
        self._abi("hftlob_rollout_prepare", int(n_slices))

    def _key_scratch(self) -> torch.Tensor:
        """Device scratch of the rollout's per-slice key chains, one per (env, caller stream)."""
        s = torch.cuda.current_stream(self.device).cuda_stream
        cache = self.__dict__.setdefault("_kscr", {})
        if s not in cache:
            cache[s] = torch.zeros(16, dtype=torch.int32, device=self.device)
        return cache[s]

    def rollout_sampled(self, key_in: torch.Tensor, key_out: torch.Tensor, state: MultiAgentState,
                        params: MultiAgentParams, n_steps: int, per_step: bool = False,
                        actions_out: Optional[torch.Tensor] = None, n_slices: Optional[int] = None,
                        key_e0: int = 0, key_n: Optional[int] = None):
        """Speed_test's whole ``rollout`` scan (Speed_test.py:186-196): bit for bit
        ``n_steps`` calls of :meth:`step_sampled` with ``key_out`` fed back as ``key_in``,
        enqueued on the current stream without host synchronisation.  The envs run as
        ``n_slices`` contiguous slices on streams of their own, so one slice's slow envs
        overlap the others' next steps.  ``key_out`` receives the master key after the
        n_steps splits.
        per_step=False: the outputs are the last step's (the scan discards them);
        per_step=True: obs / rewards / dones (and ``actions_out``, int32
        [n_steps, E, action_words] if given) carry a leading [n_steps] dimension
        (the info dict, when enabled, is flattened to [n_steps * E, ...])."""
        E = state.buf.shape[0]
        if n_steps < 1:
            raise ValueError("n_steps must be >= 1")
        if n_slices is None:
            n_slices = self.default_slices(E)
        if per_step:
            o = self._alloc((n_steps, E))
            shape = (n_steps, E, self.action_words)
        else:
            o = self._outputs(E)
            shape = (E, self.action_words)
        if actions_out is not None and (tuple(actions_out.shape) != shape or actions_out.dtype != torch.int32):
            raise ValueError(f"actions_out must be int32 {list(shape)}")
        self._abi("hftlob_env_rollout_sampled", C.byref(self.cfg_c), E, int(key_e0),
                  int(E if key_n is None else key_n), n_steps, _lib.ptr(key_in), _lib.ptr(key_out),
                  _lib.ptr(self._key_scratch()) if n_slices else None,  # (the persistent launch needs none)
                  _lib.ptr(actions_out), _lib.ptr(params.loaded_params.message_data),
                  _lib.ptr(params.loaded_params.init_states_array), _lib.ptr(state.buf), C.byref(o["struct"]),
                  int(per_step), int(n_slices))
        if not per_step:
            return self._results(o, state, E)
        T = n_steps
        flat = {k: (v.reshape((T * E,) + tuple(v.shape[2:])) if isinstance(v, torch.Tensor) else v)
                for k, v in o.items()}
        obs, _, rewards, dones, info = self._results(flat, state, T * E)
        unf = lambda x: x.reshape((T, E) + tuple(x.shape[1:]))  # noqa: E731
        obs = [unf(x) for x in obs]
        rewards = [unf(x) for x in rewards]
        dones = {"__all__": unf(dones["__all__"]), "agents": [unf(x) for x in dones["agents"]]}
        return obs, state, rewards, dones, info

    def _results(self, o, state, E):
        self.last_info_words = o["info"]  # raw info record of the last step (int32 [E, info_words]) or None
        obs, a = self._split_types(o["obs"], True), 0
        for t, n_t in enumerate(self.multi_agent_config.number_of_agents_per_type):
            obs[t] = self._message_obs(o, obs[t], t, a, n_t, E)
            a += n_t
        rewards = self._split_types(o["rewards"], False)
        dones = {"__all__": o["done_all"], "agents": self._split_types(o["dones"], False)}
        return obs, state, rewards, dones, self._info(o, E)

    def sample_actions(self, key: torch.Tensor) -> torch.Tensor:
        """Speed_test.py:166-177 random actions on device: int32 [E, action_words]
        (== [E, num_agents] unless an agent type has a MultiDiscrete space)."""
        keys = self._keys(key)
        acts = torch.empty((keys.shape[0], self.action_words), dtype=torch.int32, device=self.device)
        self._abi("hftlob_sample_actions", C.byref(self.cfg_c), keys.shape[0], _lib.ptr(keys), _lib.ptr(acts))
        return acts


def split_keys(keys: torch.Tensor, n: int, partitionable: bool = True) -> torch.Tensor:
    """jax.random.split per row: uint32 [E, 2] -> [E, n, 2] (device)."""
    keys = keys.contiguous()
    out = torch.empty((keys.shape[0], n, 2), dtype=keys.dtype, device=keys.device)
    with torch.cuda.device(keys.device):
        _lib.check(_lib.lib().hftlob_split_keys(keys.shape[0], n, int(partitionable), _lib.ptr(keys), _lib.ptr(out),
                                                _lib.stream_ptr(device=keys.device)))
    return out
