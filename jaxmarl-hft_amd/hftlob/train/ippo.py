"""IPPO with recurrent actor-critics, trained against the HIP env step (the
reference's consumer loop, gymnax_exchange/jaxrl/MARL/ippo_rnn_JAXMARL.py).

One network (and optimizer) per agent type, as the reference:

* ``ActorCriticRNN`` (:203-256): Dense(FC_DIM_SIZE, orthogonal sqrt 2) + relu ->
  GRU(GRU_HIDDEN_DIM) whose carry is zeroed where the actor's previous done is set
  (ScannedRNN, :53-78) -> critic Dense(FC)+relu+Dense(1) and actor
  Dense(GRU_HIDDEN_DIM)+relu+Dense(n_actions, orthogonal 0.01) categorical head
  (SingleActionOutput :183-201).
* rollout (:578-663): NUM_STEPS steps of sample -> env.step, the transitions kept
  in preallocated device buffers (no host synchronisation inside the rollout);
  actors are (env, agent) pairs of one type, ``batchify`` order.
* GAE (:668-690) with the per-type GAMMA / GAE_LAMBDA and the env's global done.
* PPO update (:711-838): UPDATE_EPOCHS x NUM_MINIBATCHES over a permutation of
  the actors (whole sequences, the GRU is re-run from the rollout's initial carry);
  clipped value loss, clipped surrogate with per-minibatch advantage
  normalisation, entropy bonus; Adam(eps 1e-5) after global-norm clipping, linear
  LR annealing by update count.
* multi-GPU (ippo_rnn_JAXMARL_pmap.py:566-567 pmean of grads): every rank steps
  its own env shard; gradients are averaged with one all-reduce per agent type
  and minibatch (``torch.distributed``, RCCL on ROCm).

On the GPU each minibatch step (forward over the sequence, loss, backward,
clipping, Adam) is captured once per agent type in a HIP graph and replayed
(``CUDA_GRAPHS``, single-process runs): a 64-step GRU unroll is thousands of small
kernels, and replaying them as one graph removes their launch cost.

Differences that are not semantics of the env: action sampling and parameter
initialisation draw from torch's generator, not JAX's threefry, and the network
runs through torch (rocBLAS GEMMs) rather than XLA.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..env import MARLEnv, split_keys


def _per_type(v, n: int) -> list:
    """A per-agent-type hyper-parameter list of length n (a scalar or a shorter list repeats its last value)."""
    v = list(v) if isinstance(v, (list, tuple)) else [v]
    return (v + [v[-1]] * n)[:n]


def default_config(**kw) -> Dict:
    """The reference's ippo_rnn_JAXMARL_2player.yaml hyper-parameters (training keys only)."""
    c = {"LR": [2.5e-4, 2.5e-4], "NUM_ENVS": 4096, "NUM_STEPS": 64, "GRU_HIDDEN_DIM": 256, "FC_DIM_SIZE": 256,
         "TOTAL_TIMESTEPS": 5e8, "UPDATE_EPOCHS": 4, "NUM_MINIBATCHES": 4, "GAMMA": [0.999999999, 0.999],
         "GAE_LAMBDA": [0.85, 0.9], "CLIP_EPS": 0.2, "ENT_COEF": [0.01, 0.01], "VF_COEF": [0.5, 0.5],
         "MAX_GRAD_NORM": [0.5, 0.5], "ANNEAL_LR": [True, True], "NUM_AGENTS_PER_TYPE": [1, 1], "SEED": 2,
         "CUDA_GRAPHS": True}
    c.update(kw)
    return c


class ActorCriticRNN(nn.Module):
    def __init__(self, obs_dim: int, n_actions: int, fc: int, hidden: int):
        super().__init__()
        self.embed = nn.Linear(obs_dim, fc)
        self.gru = nn.GRUCell(fc, hidden)
        self.critic1, self.critic2 = nn.Linear(hidden, fc), nn.Linear(fc, 1)
        self.actor1, self.actor2 = nn.Linear(hidden, hidden), nn.Linear(hidden, n_actions)
        for m, g in ((self.embed, math.sqrt(2)), (self.critic1, 2.0), (self.critic2, 1.0), (self.actor1, 2.0),
                     (self.actor2, 0.01)):
            nn.init.orthogonal_(m.weight, g)
            nn.init.zeros_(m.bias)
        self.hidden = hidden

    def step(self, h: torch.Tensor, obs: torch.Tensor, done: torch.Tensor):
        """One time step for a batch of actors: (new carry, logits, value)."""
        h = torch.where(done[:, None], torch.zeros_like(h), h)
        h = self.gru(F.relu(self.embed(obs)), h)
        v = self.critic2(F.relu(self.critic1(h))).squeeze(-1)
        return h, self.actor2(F.relu(self.actor1(h))), v

    def forward(self, h0: torch.Tensor, obs: torch.Tensor, dones: torch.Tensor):
        """A sequence [T, B, ...] from carry h0 (the ScannedRNN scan): logits [T, B, A], values [T, B].
        The same cell as ``step``; the input-side GEMMs (embedding, the GRU's input
        projection, both heads) run once over all T, only h @ W_hh stays in the scan."""
        # unbind / chunk (not slicing): their backward concatenates the per-step grads once,
        # where a slice's backward would zero-fill and add a whole [T, B, 3H] grad per step
        gis = F.linear(F.relu(self.embed(obs)), self.gru.weight_ih, self.gru.bias_ih).unbind(0)  # (r, z, n)
        w_hh, b_hh = self.gru.weight_hh, self.gru.bias_hh
        h = h0
        hs = []
        for t, gi in enumerate(gis):
            h = torch.where(dones[t][:, None], torch.zeros_like(h), h)
            ir, iz, i_n = gi.chunk(3, -1)
            hr, hz, hn = F.linear(h, w_hh, b_hh).chunk(3, -1)
            r = torch.sigmoid(ir + hr)
            z = torch.sigmoid(iz + hz)
            n = torch.tanh(i_n + r * hn)
            h = (1.0 - z) * n + z * h
            hs.append(h)
        hseq = torch.stack(hs)
        return self.actor2(F.relu(self.actor1(hseq))), self.critic2(F.relu(self.critic1(hseq))).squeeze(-1)


@dataclass
class Rollout:
    """One agent type's trajectory buffers, [T, n_actors, ...] on the device."""
    obs: torch.Tensor
    done: torch.Tensor          # the actor's done entering the step (GRU reset)
    global_done: torch.Tensor   # dones["__all__"] of the env (GAE)
    action: torch.Tensor
    value: torch.Tensor
    reward: torch.Tensor
    log_prob: torch.Tensor


def calculate_gae(reward, value, global_done, last_val, gamma: float, lam: float):
    """_calculate_gae (:668-690): reverse scan; returns (advantages, targets)."""
    T = reward.shape[0]
    adv = torch.empty_like(reward)
    gae = torch.zeros_like(last_val)
    next_value = last_val
    for t in range(T - 1, -1, -1):
        nd = 1.0 - global_done[t].to(reward.dtype)
        delta = reward[t] + gamma * next_value * nd - value[t]
        gae = delta + gamma * lam * nd * gae
        adv[t] = gae
        next_value = value[t]
    return adv, adv + value


def ppo_loss(logits, values, rb_action, rb_value, rb_log_prob, gae, targets, clip_eps: float, vf_coef: float,
             ent_coef: float):
    """_loss_fn (:718-765) -> (total, value_loss, actor_loss, entropy, approx_kl, clip_frac)."""
    logp_all = F.log_softmax(logits, -1)
    log_prob = logp_all.gather(-1, rb_action.long().unsqueeze(-1)).squeeze(-1)
    v_clip = rb_value + (values - rb_value).clamp(-clip_eps, clip_eps)
    value_loss = 0.5 * torch.maximum((values - targets) ** 2, (v_clip - targets) ** 2).mean()
    logratio = log_prob - rb_log_prob
    ratio = torch.exp(logratio)
    gae = (gae - gae.mean()) / (gae.std(unbiased=False) + 1e-8)
    actor_loss = -torch.minimum(ratio * gae, ratio.clamp(1.0 - clip_eps, 1.0 + clip_eps) * gae).mean()
    entropy = -(logp_all.exp() * logp_all).sum(-1).mean()
    approx_kl = ((ratio - 1) - logratio).mean()
    clip_frac = ((ratio - 1).abs() > clip_eps).float().mean()
    total = actor_loss + vf_coef * value_loss - ent_coef * entropy
    return total, value_loss, actor_loss, entropy, approx_kl, clip_frac


def linear_schedule(lr: float, count: int, n_minibatches: int, n_epochs: int, n_updates: int) -> float:
    """linear_schedule (:503-509): lr * (1 - (count // (minibatches * epochs)) / NUM_UPDATES)."""
    return lr * (1.0 - (count // (n_minibatches * n_epochs)) / n_updates)


def _average_grads(params, dist) -> None:
    """pmean of the gradients over ranks: one flattened all-reduce (bucket) per call."""
    grads = [p.grad for p in params if p.grad is not None]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    flat /= dist.get_world_size()
    o = 0
    for g in grads:
        g.copy_(flat[o:o + g.numel()].view_as(g))
        o += g.numel()


class IPPOTrainer:
    """make_train(config)(rng) of the reference, one ``update`` per call."""

    def __init__(self, env: MARLEnv, config: Dict, dist=None, device=None):
        self.env, self.c, self.dist = env, config, dist
        self.device = torch.device(device or env.device)
        nt = len(env.list_of_agents_configs)
        self.n_types = nt
        c = config
        for k in ("LR", "GAMMA", "GAE_LAMBDA", "ENT_COEF", "VF_COEF", "MAX_GRAD_NORM", "ANNEAL_LR"):
            c[k] = _per_type(c[k], nt)
        # NUM_ENVS is global, as in the reference's pmap learner: each of the N ranks steps
        # NUM_ENVS // N envs, NUM_UPDATES = TOTAL_TIMESTEPS // NUM_STEPS // NUM_ENVS
        # (ippo_rnn_JAXMARL_pmap.py:209-211, 329-332, 419)
        world = dist.get_world_size() if dist is not None else 1
        rank = dist.get_rank() if dist is not None else 0
        n_global = int(c["NUM_ENVS"])
        if n_global % world:
            raise ValueError(f"NUM_ENVS ({n_global}) must be a multiple of the world size ({world})")
        self.E, self.T = n_global // world, c["NUM_STEPS"]
        self.n_agents = list(env.multi_agent_config.number_of_agents_per_type)
        self.n_actors = [n * self.E for n in self.n_agents]
        self.num_updates = max(1, int(c["TOTAL_TIMESTEPS"] // self.T // n_global))
        for i, sp in enumerate(env.action_spaces):
            if not isinstance(getattr(sp, "n", None), int):   # the categorical head is Dense(action_space.n)
                raise NotImplementedError(f"agent type {i}: IPPO-RNN needs a Discrete action space "
                                          "(ippo_rnn_JAXMARL.py ActorCriticRNN; EXE fixed_prices is MultiDiscrete)")
        torch.manual_seed(c["SEED"])  # the same initial parameters on every rank
        self.nets = [ActorCriticRNN(env.observation_spaces[i].shape[0], env.action_spaces[i].n, c["FC_DIM_SIZE"],
                                    c["GRU_HIDDEN_DIM"]).to(self.device) for i in range(nt)]
        # HIP-graph minibatch steps: single process on the GPU (the grad all-reduce stays eager)
        self.graphs = bool(c.get("CUDA_GRAPHS", False)) and self.device.type == "cuda" and world == 1
        if self.graphs:  # capturable Adam: step counter and lr live on the device
            self.opts = [torch.optim.Adam(n.parameters(), lr=torch.tensor(c["LR"][i], device=self.device), eps=1e-5,
                                          capturable=True) for i, n in enumerate(self.nets)]
        else:
            self.opts = [torch.optim.Adam(n.parameters(), lr=c["LR"][i], eps=1e-5) for i, n in enumerate(self.nets)]
        self._roll = None        # the captured rollout graph (False: not capturable, stays eager)
        self.opt_count = [0] * nt
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(c["SEED"] + 1000 * rank)
        self.params = env.default_params
        self._split = getattr(env, "split_keys", split_keys)   # device threefry split (jax.random.split)
        # rng = PRNGKey(SEED); rng, _rng = split(rng); reset keys = split(_rng, NUM_ENVS), sharded over
        # the ranks in order; each rank then draws its step keys from its own rng.  This follows the
        # SHAPE of the reference's key chain (:283-284, 329) but not its values: the reference also
        # splits rng once per agent type for the network init (:246) before the reset split, and
        # draws the per-device rngs as split(split(rng)[1], N_DEVICES) (:775-776).  The networks are
        # torch-initialised here, so the same SEED gives different reset / step keys than JAX.
        master = torch.tensor([[0, c["SEED"]]], dtype=torch.int32, device=self.device)
        k = self._split(master, 2)[0]
        self.rng = (k[0] if world == 1 else self._split(k[0:1].contiguous(), world)[0][rank]).clone()
        reset_keys = self._split(k[1:2].contiguous(), n_global)[0][rank * self.E:(rank + 1) * self.E].contiguous()
        self.reset_keys = reset_keys
        obs, self.state = env.reset(reset_keys, self.params)
        self.last_obs = [o.reshape(n, -1).clone() for o, n in zip(obs, self.n_actors)]
        self.last_done = [torch.zeros(n, dtype=torch.bool, device=self.device) for n in self.n_actors]
        self.h = [torch.zeros(n, c["GRU_HIDDEN_DIM"], device=self.device) for n in self.n_actors]
        T = self.T
        self.buf = [Rollout(obs=torch.empty((T, n, env.observation_spaces[i].shape[0]), device=self.device),
                            done=torch.empty((T, n), dtype=torch.bool, device=self.device),
                            global_done=torch.empty((T, n), dtype=torch.bool, device=self.device),
                            action=torch.empty((T, n), dtype=torch.int32, device=self.device),
                            value=torch.empty((T, n), device=self.device),
                            reward=torch.empty((T, n), device=self.device),
                            log_prob=torch.empty((T, n), device=self.device))
                    for i, n in enumerate(self.n_actors)]

    def _next_keys(self) -> torch.Tensor:
        """rng, _rng = split(rng); rng_step = split(_rng, NUM_ENVS) (:613-614)."""
        k = self._split(self.rng[None], 2)[0]
        self.rng.copy_(k[0])
        return self._split(k[1:2].contiguous(), self.E)[0].contiguous()

    @torch.no_grad()
    def rollout(self) -> None:
        """NUM_STEPS of _env_step (:578-658), all on the device; with CUDA_GRAPHS the whole
        rollout (policy, sampling, env steps, buffer writes) is one captured HIP graph."""
        if not self.graphs or self._roll is False:
            return self._rollout()
        if self._roll is None:  # one eager rollout (warm-up), then capture; capture runs nothing
            self._rollout_side()
            self._roll = 0
            return None
        if self._roll == 0:
            g = torch.cuda.CUDAGraph()
            g.register_generator_state(self.gen)
            try:
                with torch.cuda.graph(g):
                    self._rollout()
            except RuntimeError:  # an op that cannot be captured: stay eager
                self._roll = False
                return self._rollout()
            self._roll = g
        self._roll.replay()
        return None

    def _rollout_side(self) -> None:
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self._rollout()
        torch.cuda.current_stream(self.device).wait_stream(side)

    def _rollout(self) -> None:
        for t in range(self.T):
            actions = []
            for i, net in enumerate(self.nets):
                b = self.buf[i]
                b.obs[t].copy_(self.last_obs[i])
                b.done[t].copy_(self.last_done[i])
                h, logits, v = net.step(self.h[i], self.last_obs[i], self.last_done[i])
                self.h[i].copy_(h)
                probs = torch.softmax(logits, -1)
                a = torch.multinomial(probs, 1, generator=self.gen).squeeze(-1)
                b.action[t].copy_(a)
                b.value[t].copy_(v)
                b.log_prob[t].copy_(torch.log_softmax(logits, -1).gather(-1, a.unsqueeze(-1)).squeeze(-1))
                actions.append(a.view(self.E, self.n_agents[i]))
            obs, self.state, rew, dones, _ = self.env.step(self._next_keys(), self.state, actions, self.params)
            for i in range(self.n_types):
                b = self.buf[i]
                b.reward[t].copy_(rew[i].reshape(-1))
                b.global_done[t].copy_(dones["__all__"].repeat_interleave(self.n_agents[i]))
                self.last_obs[i].copy_(obs[i].reshape(self.n_actors[i], -1))
                self.last_done[i].copy_(dones["agents"][i].reshape(-1))

    def _static(self, i: int, n: int, mb: int):
        """Fixed-address inputs of agent type i's minibatch step (what a captured graph reads)."""
        if not hasattr(self, "_st"):
            self._st = [None] * self.n_types
        if self._st[i] is None:
            T, H = self.T, self.c["GRU_HIDDEN_DIM"]
            self._st[i] = {"h0": torch.empty((n, H), device=self.device),
                           "adv": torch.empty((T, n), device=self.device),
                           "tgt": torch.empty((T, n), device=self.device),
                           "idx": torch.zeros(n // mb, dtype=torch.long, device=self.device),
                           "warm": 0, "graph": None, "out": None}
        return self._st[i]

    def _mb_step(self, i: int) -> torch.Tensor:
        """One PPO minibatch step of agent type i from the static inputs: forward over the
        sequences, loss, backward, grad pmean (multi-rank), global-norm clip, Adam."""
        c, net, opt, b, st = self.c, self.nets[i], self.opts[i], self.buf[i], self._st[i]
        idx = st["idx"]
        logits, values = net(st["h0"][idx], b.obs[:, idx], b.done[:, idx])
        out = ppo_loss(logits, values, b.action[:, idx], b.value[:, idx], b.log_prob[:, idx],
                       st["adv"][:, idx], st["tgt"][:, idx], c["CLIP_EPS"], c["VF_COEF"][i], c["ENT_COEF"][i])
        out[0].backward()
        if self.dist is not None and self.dist.get_world_size() > 1:
            _average_grads(list(net.parameters()), self.dist)
        torch.nn.utils.clip_grad_norm_(net.parameters(), c["MAX_GRAD_NORM"][i])
        opt.step()
        return torch.stack([x.detach() for x in out])

    def _minibatch(self, i: int) -> torch.Tensor:
        st, opt = self._st[i], self.opts[i]
        if not self.graphs:
            opt.zero_grad(set_to_none=True)
            return self._mb_step(i)
        if st["graph"] is None and st["warm"] < 2:  # eager steps on a side stream before capture
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                opt.zero_grad(set_to_none=True)
                r = self._mb_step(i)
            torch.cuda.current_stream(self.device).wait_stream(side)
            st["warm"] += 1
            return r
        if st["graph"] is None:  # capture once (nothing runs), then replay below
            opt.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st["out"] = self._mb_step(i)
            st["graph"] = g
        st["graph"].replay()
        return st["out"].clone()

    def update(self) -> Dict:
        """One _update_step: rollout, GAE, UPDATE_EPOCHS x NUM_MINIBATCHES PPO steps per agent type."""
        c = self.c
        h0 = [h.clone() for h in self.h]
        self.rollout()
        metrics = {"loss": [], "avg_reward": []}
        for i, net in enumerate(self.nets):
            b = self.buf[i]
            n, mb = self.n_actors[i], c["NUM_MINIBATCHES"]
            st = self._static(i, n, mb)
            with torch.no_grad():
                _, _, last_val = net.step(self.h[i], self.last_obs[i], self.last_done[i])
                adv, targets = calculate_gae(b.reward, b.value, b.global_done, last_val, c["GAMMA"][i],
                                             c["GAE_LAMBDA"][i])
                st["h0"].copy_(h0[i]); st["adv"].copy_(adv); st["tgt"].copy_(targets)
            stats = torch.zeros(6, device=self.device)
            for _ in range(c["UPDATE_EPOCHS"]):
                perm = torch.randperm(n, device=self.device, generator=self.gen)
                for idx in perm.view(mb, n // mb):
                    if c["ANNEAL_LR"][i]:
                        lr = linear_schedule(c["LR"][i], self.opt_count[i], mb, c["UPDATE_EPOCHS"], self.num_updates)
                        for g in self.opts[i].param_groups:
                            if torch.is_tensor(g["lr"]):
                                g["lr"].fill_(lr)
                            else:
                                g["lr"] = lr
                    st["idx"].copy_(idx)
                    stats += self._minibatch(i)
                    self.opt_count[i] += 1
            stats /= c["UPDATE_EPOCHS"] * mb
            metrics["loss"].append(dict(zip(("total_loss", "value_loss", "actor_loss", "entropy", "approx_kl",
                                             "clip_frac"), stats)))
            metrics["avg_reward"].append(b.reward.mean())
        return metrics


def train(env: MARLEnv, config: Dict, n_updates: Optional[int] = None, dist=None, log=print):
    """Runs ``n_updates`` (default NUM_UPDATES) updates; returns (trainer, env-steps/s over the run)."""
    tr = IPPOTrainer(env, config, dist=dist)
    n = n_updates or tr.num_updates
    sync = torch.cuda.synchronize if tr.device.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    for u in range(n):
        m = tr.update()
        if log is not None:
            log({"update": u, "avg_reward": [float(r) for r in m["avg_reward"]],
                 "loss": [{k: float(v) for k, v in d.items()} for d in m["loss"]]})
    sync()
    world = dist.get_world_size() if dist is not None else 1
    return tr, n * tr.T * tr.E * world / (time.perf_counter() - t0)   # E * world = NUM_ENVS


def main(argv=None) -> None:
    """python -m hftlob.train.ippo [--rl-config ippo.yaml] [--env-config 2_player_fq_fqc] [--updates N]"""
    import argparse
    import json
    import yaml
    from ..config_io import builtin_config, load_config_from_file
    ap = argparse.ArgumentParser()
    ap.add_argument("--rl-config", default=None, help="reference-style YAML (ippo_rnn_JAXMARL_2player.yaml keys)")
    ap.add_argument("--env-config", default="2_player_fq_fqc", help="JSON path or builtin config name")
    ap.add_argument("--updates", type=int, default=2)
    ap.add_argument("--envs", type=int, default=None)
    ap.add_argument("--data", default=None, help="'lobster' to load world_config.dataPath (else synthetic)")
    a = ap.parse_args(argv)
    c = default_config()
    if a.rl_config:
        with open(a.rl_config) as f:
            c.update({k: v for k, v in yaml.safe_load(f).items() if k in c})
    if a.envs:
        c["NUM_ENVS"] = a.envs
    cfg = (load_config_from_file(a.env_config) if a.env_config.endswith((".json", ".yaml"))
           else builtin_config(a.env_config))
    env = MARLEnv(None, cfg, data=a.data, return_info=False, persistent_outputs=True)
    _, sps = train(env, c, a.updates, log=lambda m: print(json.dumps(m)))
    print(json.dumps({"env_steps_per_s_incl_learner": sps, "num_envs": c["NUM_ENVS"], "num_steps": c["NUM_STEPS"]}))


if __name__ == "__main__":
    main()
