"""``PPOEngine`` -- drop-in for the reference ``PPO`` algorithm (ppo.py:11-159, base_algorithm.py:14-61).

Same surface: ``PPOEngine(environment_helper, agent)``, ``iterate()`` -> ``_iterate()`` ->
``rollout()`` (returns the buffer), ``calculate_advantages(memory)`` (adds ``advantage`` and
``current_state_value_target``), ``train(memory)``.  The Python here only sequences launches; all
arithmetic runs in the engine's HIP kernels on the current stream, and the host reads back once
per iteration (losses, mean reward) instead of twice per minibatch (ppo.py:139-140).

RNG (``Run.engine_config.rng``):
  "torch"  -- the reference's draws from the torch global CPU generator, in its order: per rollout
              step one (N, A) ``Normal.sample`` (ppo.py:23-25), per epoch ``randperm(N*T)``
              (ppo.py:103) and per minibatch the (B, A) sample that ppo.py:110 draws and drops.
  "philox" -- on-device Philox normals and a keyed Feistel permutation (no host RNG, no H2D).
Data parallel (``dist`` = torch.distributed initialised, backend RCCL): each rank owns its env
shard; per optimizer step ONE all-reduce(SUM) of the flat actor+critic gradient, with every rank
scaling its loss by the global minibatch size.
"""
from __future__ import annotations

import time
import warnings
from typing import Callable, Optional

import torch

from . import engine as E
from .buffer import RolloutBuffer
from .distributed import DataParallel
from .features import Run


def _default_log(msg: str) -> None:
    print(msg, flush=True)


class PPOEngine:
    def __init__(self, environment_helper, agent, log: Optional[Callable[[str], None]] = None,
                 process_group=None):
        self.environment_helper = environment_helper
        self.agent = agent
        self.run: Run = environment_helper.run
        self.log = log or _default_log
        self.dp = DataParallel(process_group, mode=getattr(self.run.engine_config, "dp_mode",
                                                           "local"))
        self.world = self.dp.world
        self.dp.broadcast_params(agent.flat_params)  # every replica starts from rank 0's params
        eng = getattr(agent, "engine", None)
        if eng is not None:  # native RCCL communicator on the ctx (RCCL groups), logged-loss share
            self.dp.attach(eng, agent.device)
        agent._algorithm = self  # agent.save / load carry the per-rank generator (engine_rng_rank*.pth)
        self.set_rng_state(getattr(agent, "_loaded_rng_state", None))  # agent.load() before us
        agent._loaded_rng_state = None
        ec, nc = self.run.environment_config, self.run.network_config
        if hasattr(agent, "make_buffer"):  # agents with their own state storage (u8 frames)
            self.buffer = agent.make_buffer(ec.num_envs, ec.maximum_timesteps)
        else:
            self.buffer = RolloutBuffer(ec.num_envs, ec.maximum_timesteps, nc.input_shape,
                                        ec.window_length, nc.output_shape, agent.device)
        self.iteration = 0
        self.last_losses = (float("nan"), float("nan"))
        self.last_mean_reward = float("nan")
        self.timings = {}
        self._rows = None
        self._count = None
        self._loss_buf = None
        self._graph = None        # captured rollout (philox + graph_safe helper)
        self._graph_warm = False
        self._rng_counter = None

    # ---- helpers -----------------------------------------------------------------------------
    def _rng(self) -> str:
        return self.run.engine_config.rng

    def _seed(self) -> int:
        return int(self.run.engine_config.seed)

    def _eps(self, n: int, a: int):
        """(eps tensor or None, philox offset) for one (n, A) sampling draw.  In exact data
        parallel mode every rank draws the GLOBAL (N, A) normals and keeps its shard's rows, so
        the sharded run consumes the reference RNG stream exactly like one process."""
        if self._rng() == "torch":
            if self.dp.world > 1 and self.dp.mode == "exact":
                lo, hi = self.dp.my_shard(n)
                eps = torch.randn(self.dp.global_envs(n), a)[lo:hi]
            else:
                eps = torch.randn(n, a, generator=self._local_gen())
            return eps.to(self.agent.device, non_blocking=True), 0
        return None, None

    def _local_gen(self):
        """Generator for the torch-RNG draws: the global CPU generator (the reference's stream)
        except in local data-parallel mode, where every rank starts from the same seeded
        parameters and would otherwise draw identical noise and row orders on every env shard;
        there each rank forks its own generator.  Its key mixes the user's global seed
        (torch.initial_seed(), so torch.manual_seed changes the run), the engine seed and the
        rank; it is a CPU Mersenne-Twister stream, independent of the device Philox key
        (seed * 1_000_003 + 17 + 7919 * rank) that only keys counter-based rollout noise.  Its
        state is checkpointed by agent.save() (engine_rng.pth) and restored by agent.load()."""
        if not (self.dp.world > 1 and self.dp.mode == "local"):
            return None
        if getattr(self, "_rank_gen", None) is None:
            key = (torch.initial_seed() * 1_000_003 + self._seed() * 7_919_993
                   + 7919 * (self.dp.rank + 1)) % (1 << 63)
            self._rank_gen = torch.Generator().manual_seed(key)
            if getattr(self, "_pending_rng_state", None) is not None:
                self._rank_gen.set_state(self._pending_rng_state)
                self._pending_rng_state = None
        return self._rank_gen

    def rng_state(self) -> Optional[dict]:
        """The per-rank generator's state (local data-parallel torch-RNG runs), for checkpoints."""
        gen = getattr(self, "_rank_gen", None)
        return None if gen is None else {"rank": self.dp.rank, "state": gen.get_state()}

    def set_rng_state(self, state: Optional[dict]) -> None:
        if not state:
            return
        if state.get("rank") != self.dp.rank:
            raise ValueError(f"engine_rng.pth holds rank {state.get('rank')}'s generator, "
                             f"this is rank {self.dp.rank}")
        gen = getattr(self, "_rank_gen", None)
        if gen is None:
            self._pending_rng_state = state["state"]
        else:
            gen.set_state(state["state"])

    # ---- ppo.py:13-60 ----------------------------------------------------------------------
    def _graph_ok(self) -> bool:
        return (self._rng() == "philox" and hasattr(self.agent.engine, "set_rng_counter") and
                bool(getattr(self.run.engine_config, "rollout_graph", False)) and
                bool(getattr(self.environment_helper, "graph_safe", False)) and
                bool(getattr(self.environment_helper, "writes_into_buffer", False)))

    @torch.no_grad()
    def rollout(self) -> RolloutBuffer:
        buf = self.buffer
        n, t_len, a = buf.num_envs, buf.horizon, buf.act_dim
        if not self._graph_ok():
            return self._rollout_steps(base_off=self.iteration * (t_len * n * a))
        # hipGraph path: the Philox offset base lives in a device counter that the policy head
        # reads at run time, so one captured T-step rollout replays with fresh noise; the
        # sampled values are identical to the eager path (offset = base + t*N*A either way).
        eng = self.agent.engine
        if self._rng_counter is None:
            self._rng_counter = torch.zeros(1, dtype=torch.int64, device=self.agent.device)
            eng.set_rng_counter(self._rng_counter)
        self._rng_counter.fill_(self.iteration * (t_len * n * a))
        if self._graph is None:
            if not self._graph_warm:  # first call eager: lazy allocations happen outside capture
                self._graph_warm = True
                return self._rollout_steps(base_off=0)
            torch.cuda.synchronize(self.agent.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._rollout_steps(base_off=0)
            self._graph = g
        self._graph.replay()
        self.environment_helper.t = t_len  # the host-side step counter the replay skipped
        return buf

    def _rollout_fused(self, base_off: int) -> RolloutBuffer:
        """Rollout through ppo_observe_act: per step one env launch (helper.step_raw) and one
        engine launch (window push + standardisation + actor/critic + sampling); same values as
        the step / get_state / policy_step sequence below."""
        helper, eng, buf = self.environment_helper, self.agent.engine, self.buffer
        n, t_len, a = buf.num_envs, buf.horizon, buf.act_dim
        helper.reset()
        helper.reset_environment(test_phase=False)
        eng.pack_weights()
        window = helper.timestep.observation
        norm = bool(self.run.normalize_observations)
        seed = self._seed() * 1_000_003 + 17 + 7919 * self.dp.rank
        noise = None
        if self._rng() == "philox" and getattr(eng, "fused", False):
            # the whole rollout's Philox noise in one launch ahead of the steps (bitwise the
            # in-kernel draws: index base_off [+ the device counter] + t*N*A + env*A + a), so the
            # policy kernel loads it with the observations instead of computing it on its
            # critical path
            if getattr(self, "_noise", None) is None or self._noise.shape != (t_len, n, a):
                self._noise = torch.empty(t_len, n, a, device=self.agent.device)
            noise = self._noise
            E.philox_normal(seed, base_off, noise, counter=getattr(eng, "_rng_counter", None))
        eps = noise[0] if noise is not None else self._eps(n, a)[0]
        eng.observe_act(window, buf.states[0], normalize=norm, eps=eps, seed=seed,
                        offset=base_off, action=buf.actions[0], logp=buf.logp[0],
                        value=buf.values[0])
        for t in range(t_len):
            obs = helper.step_raw(buf.actions[t], buf.reward[t], buf.terminated[t])
            if t + 1 < t_len:
                eps = noise[t + 1] if noise is not None else self._eps(n, a)[0]
                eng.observe_act(window, buf.states[t + 1], obs=obs, reset=buf.terminated[t],
                                normalize=norm, eps=eps, seed=seed,
                                offset=base_off + (t + 1) * n * a, action=buf.actions[t + 1],
                                logp=buf.logp[t + 1], value=buf.values[t + 1])
            else:
                eng.observe_act(window, buf.states[t_len], obs=obs, reset=buf.terminated[t],
                                normalize=norm, value=buf.values[t_len])
        return buf

    def _rollout_pipelined(self, base_off: int) -> RolloutBuffer:
        """Rollout over a host-physics helper split into halves (HostPhysicsVecEnvHelper,
        overlap=True): per step and half, the half's observe + act (ppo_observe_act on its rows,
        Philox offsets / eps rows of the full step, so the values equal the unsplit rollout), its
        action D2H on its side stream, its workers' physics and its H2D uploads.  The host
        releases each half as soon as its actions land, so one half's physics runs while the GPU
        computes the other half's policy step (running_gym_sequential_vectorized.py:40-59 is the
        serial reference loop)."""
        helper, eng, buf = self.environment_helper, self.agent.engine, self.buffer
        n, t_len, a = buf.num_envs, buf.horizon, buf.act_dim
        helper.reset()
        helper.reset_environment(test_phase=False)
        eng.pack_weights()
        window = helper.timestep.observation
        norm = bool(self.run.normalize_observations)
        seed = self._seed() * 1_000_003 + 17 + 7919 * self.dp.rank
        halves = helper.halves
        if hasattr(eng, "host_rollout") and hasattr(helper, "native_desc"):
            # the whole T-step pipeline in one native call (csrc/host_rollout.hip); the noise of
            # every step is drawn up front in the same order as the per-step draws below
            eps = None
            if self._rng() == "torch":
                eps = torch.empty(t_len, n, a, device=self.agent.device)
                for t in range(t_len):
                    eps[t].copy_(self._eps(n, a)[0])
            desc = helper.native_desc()
            eng.host_rollout(desc, window, norm, buf.states, buf.actions, buf.logp, buf.values,
                             buf.reward, buf.terminated, helper._obs_next, eps, seed, base_off)
            helper.native_done(desc, buf.reward[t_len - 1], buf.terminated[t_len - 1])
            return buf

        def act(t, obs_rows=None, reset_rows=None, eps=None, g=0, last=False):
            lo, hi = halves[g]
            rows = slice(lo, hi)
            if last:
                eng.observe_act(window[rows], buf.states[t][rows], obs=obs_rows, reset=reset_rows,
                                normalize=norm, value=buf.values[t][rows])
                return
            eng.observe_act(window[rows], buf.states[t][rows], obs=obs_rows, reset=reset_rows,
                            all_reset=False, normalize=norm,
                            eps=None if eps is None else eps[rows], seed=seed,
                            offset=base_off + t * n * a + lo * a, action=buf.actions[t][rows],
                            logp=buf.logp[t][rows], value=buf.values[t][rows])
            helper.begin_half(g, buf.actions[t][rows])

        eps, _ = self._eps(n, a)
        for g in range(len(halves)):
            act(0, eps=eps, g=g)
        for t in range(t_len):
            for g in range(len(halves)):
                helper.release_half(g, t)
            if t + 1 < t_len:
                eps, _ = self._eps(n, a)
            for g, (lo, hi) in enumerate(halves):
                obs = helper.finish_half(g, buf.reward[t][lo:hi], buf.terminated[t][lo:hi])
                act(t + 1, obs, buf.terminated[t][lo:hi], eps, g, last=t + 1 == t_len)
            helper.end_step(buf.reward[t], buf.terminated[t])
        return buf

    def _rollout_steps(self, base_off: int) -> RolloutBuffer:
        helper, eng, buf = self.environment_helper, self.agent.engine, self.buffer
        n, t_len, a = buf.num_envs, buf.horizon, buf.act_dim
        if len(getattr(helper, "halves", ())) > 1 and \
                getattr(self.run.engine_config, "fused_rollout", True):
            return self._rollout_pipelined(base_off)
        if hasattr(helper, "step_raw") and getattr(self.run.engine_config, "fused_rollout", True):
            return self._rollout_fused(base_off)
        helper.reset()
        helper.reset_environment(test_phase=False)
        # helpers that can write straight into the buffer (SyntheticVecEnvHelper) skip the copies
        fast_state = fast_step = bool(getattr(helper, "writes_into_buffer", False))

        def observe(slot: int):
            if fast_state:
                helper.get_state(test_phase=False, out=buf.states[slot])
            else:
                buf.states[slot].copy_(helper.get_state(test_phase=False).reshape(n, -1))

        seed = self._seed() * 1_000_003 + 17 + 7919 * self.dp.rank
        observe(0)
        eps, _ = self._eps(n, a)
        eng.policy_step(buf.states[0], eps=eps, seed=seed, offset=base_off, action=buf.actions[0],
                        logp=buf.logp[0], value=buf.values[0])
        for t in range(t_len):
            if fast_step:
                helper.step(buf.actions[t], reward_out=buf.reward[t], terminated_out=buf.terminated[t])
            else:
                helper.step(buf.actions[t])
                ts = helper.environment.timestep
                buf.reward[t].copy_(torch.as_tensor(ts.reward))
                buf.terminated[t].copy_(torch.as_tensor(ts.terminated))
                buf.truncated[t].copy_(torch.as_tensor(ts.truncated))
            observe(t + 1)
            if t + 1 < t_len:
                eps, _ = self._eps(n, a)
                eng.policy_step(buf.states[t + 1], eps=eps, seed=seed,
                                offset=base_off + (t + 1) * n * a, action=buf.actions[t + 1],
                                logp=buf.logp[t + 1], value=buf.values[t + 1])
            else:
                eng.policy_step(buf.states[t_len], value=buf.values[t_len])
        return buf

    # ---- ppo.py:62-91 ----------------------------------------------------------------------
    @torch.no_grad()
    def calculate_advantages(self, memory: RolloutBuffer) -> None:
        run = self.run
        buf = memory
        t_len = buf.horizon
        rewards = buf.reward
        if run.normalize_rewards:
            if buf.reward_work is None:
                buf.reward_work = torch.empty_like(buf.reward)
            buf.reward_work.copy_(buf.reward)
            E.normalize_rows(buf.reward_work, run.ppo_config.advantage_scaler)
            rewards = buf.reward_work
        eng = getattr(self.agent, "engine", None)
        buf.records_staged = False
        if (not run.ppo_config.normalize_advantage and getattr(eng, "fused", False)
                and hasattr(eng, "gae_stage_records")):
            # fused bf16 path: the scan also writes the 128 B row records the epochs gather
            # (byte-identical to gae + stage_records; train() then skips its staging pass)
            eng.gae_stage_records(buf.values[:t_len], buf.values[1:], rewards, buf.terminated,
                                  run.ppo_config.gamma, run.ppo_config.lmbda, buf.advantage,
                                  buf.value_target, buf.states, buf.actions, buf.logp,
                                  force_last_done=True)
            buf.records_staged = True
            return
        E.gae(buf.values[:t_len], buf.values[1:], rewards, buf.terminated, run.ppo_config.gamma,
              run.ppo_config.lmbda, buf.advantage, buf.value_target, force_last_done=True)
        if run.ppo_config.normalize_advantage:
            E.normalize_rows(buf.advantage, run.ppo_config.advantage_scaler)
            E.normalize_rows(buf.value_target, run.ppo_config.advantage_scaler)

    # ---- ppo.py:93-154 ---------------------------------------------------------------------
    def _scheduled_ok(self) -> bool:
        return self._rng() == "philox" and (self.dp.world == 1 or self.dp.mode == "local")

    def _train_scheduled(self, memory: RolloutBuffer, b: int, epochs: int, batches: int, clip_lo,
                         clip_hi, inv_b, inv_ba):
        """The E x M optimizer steps of a single-rank philox iteration with everything known up
        front: the minibatch rows of every epoch are drawn first (E Feistel launches) and the Adam
        step sizes come from a device schedule.  Per step: on the fused bf16 path one
        ppo_update_step_staged (fused forward/backward + a tail that reduces, steps Adam, refreshes
        the weight images and gathers the next minibatch's rows); otherwise minibatch_grad +
        adam_sched.  Data parallel ("local" mode): the fused gradient, the all-reduce, then
        Adam + weight images + the next minibatch's gather (adam_pack(next_rows=...)).  With
        engine_config.train_graph (single rank) the loop is captured once as a hipGraph and
        replayed (same launches, bit-identical results)."""
        agent, eng, buf = self.agent, self.agent.engine, memory
        n, t_len = buf.num_envs, buf.horizon
        dev = agent.device
        steps = epochs * batches
        sched = agent.adam_schedule(steps)
        if sched is None:
            return None
        beta1, beta2 = agent.optimizers["actor"].param_groups[0]["betas"]
        eps = agent.optimizers["actor"].param_groups[0]["eps"]
        ppo = self.run.ppo_config
        # every scalar the captured graph bakes in (the step sizes live in the device schedule)
        key = (b, epochs, batches, float(clip_lo), float(clip_hi), float(ppo.entropy_eps),
               float(inv_b), float(inv_ba), float(beta1), float(beta2), float(eps), eng.fused,
               eng.precision)
        if getattr(self, "_tg_key", None) != key:
            self._tg_key = key
            self._tg_rows = torch.empty(epochs, batches * b, dtype=torch.int32, device=dev)
            self._tg_sched = torch.empty(steps, 4, dtype=torch.float32, device=dev)
            self._tg_graph = None
            self._tg_warm = False
        for epoch in range(epochs):
            E.feistel_rows(self._seed() + 7919 * self.dp.rank, self.iteration * epochs + epoch, 0,
                           batches * b, n, t_len, self._tg_rows[epoch])
        self._tg_sched.copy_(sched, non_blocking=True)

        staged = eng.fused
        if staged and not getattr(buf, "records_staged", False):
            eng.stage_records(buf.states, buf.actions, buf.logp, buf.advantage, buf.value_target)
        buf.records_staged = False

        def rows_of(k):
            e, i = divmod(k, batches)
            return self._tg_rows[e, i * b:(i + 1) * b]

        def body():
            for epoch in range(epochs):
                for i in range(batches):
                    k = epoch * batches + i
                    rows = rows_of(k)
                    sched = self._tg_sched[k]
                    nxt = rows_of(k + 1) if k + 1 < steps else None
                    if staged and self.dp.active:
                        # fused gradient (folded to the flat gradient) -> all-reduce -> ONE tail
                        # launch: Adam + weight images + the next minibatch's row gather
                        eng.minibatch_grad_staged(rows, b, agent.flat_grad, self._loss_buf[epoch, i],
                                                  clip_lo, clip_hi, ppo.entropy_eps, inv_b, inv_ba,
                                                  weights_current=k > 0, rows_gathered=k > 0)
                        if self.dp.comm is not None:  # ppo_allreduce_grads: the ctx's comm
                            eng.allreduce_grads(agent.flat_grad)
                        else:
                            self.dp.allreduce_grad(agent.flat_grad)
                        eng.adam_pack(agent.flat_grad, agent.flat_m, agent.flat_v, sched,
                                      one_minus_beta1=1 - beta1, beta2=beta2,
                                      one_minus_beta2=1 - beta2, eps=eps, next_rows=nxt)
                        continue
                    if staged:
                        eng.update_step_staged(
                            rows, b, agent.flat_grad, self._loss_buf[epoch, i], agent.flat_m,
                            agent.flat_v, clip_lo, clip_hi, ppo.entropy_eps, inv_b, inv_ba,
                            sched=sched, one_minus_beta1=1 - beta1, beta2=beta2,
                            one_minus_beta2=1 - beta2, eps=eps,
                            next_rows=nxt, weights_current=k > 0, rows_gathered=k > 0)
                        continue
                    eng.minibatch_grad(buf.states, buf.actions, buf.logp, buf.advantage,
                                       buf.value_target, rows, b, agent.flat_grad,
                                       self._loss_buf[epoch, i], clip_lo, clip_hi,
                                       ppo.entropy_eps, inv_b, inv_ba)
                    self.dp.allreduce_grad(agent.flat_grad)
                    E.adam_sched(agent.flat_params, agent.flat_grad, agent.flat_m, agent.flat_v,
                                 eng.n_actor, sched, 1 - beta1, beta2, 1 - beta2, eps)

        if (self.dp.active and not self.dp.graph_safe or self.dp.rehearse and not self.dp.comm
                or not getattr(self.run.engine_config, "train_graph", True)
                or getattr(self, "_tg_capture_failed", False)):
            body()  # torch.distributed (gloo) collectives and the no-op rehearsal stay eager
            return self._loss_buf
        if self._tg_graph is None:
            if not self._tg_warm:  # first call eager: lazy workspace / timing setup outside capture
                self._tg_warm = True
                body()
                return self._loss_buf
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            # the native RCCL all-reduce (DataParallel.comm) is recorded like a kernel; its proxy
            # threads keep running during capture, so only this thread's calls are checked
            mode = "thread_local" if self.dp.comm is not None else "global"

            def capture():
                with torch.cuda.graph(g, capture_error_mode=mode):
                    body()

            # every rank agrees on the outcome (DataParallel.capture_agreed): if the capture
            # failed on ANY rank (a collective the RCCL build cannot record), all ranks leave the
            # native communicator together and run this and every later update loop eagerly over
            # torch.distributed -- the same collective sequence everywhere.  Nothing ran during
            # the capture and body() depends on no host state it changes.
            reason = self.dp.capture_agreed(capture, eng)
            if reason is not None:
                warnings.warn(f"capturing the data-parallel step with the native RCCL all-reduce "
                              f"failed ({reason}); the update loop runs eagerly on every rank")
                self._tg_capture_failed = True
                torch.cuda.synchronize(dev)
                body()
                return self._loss_buf
            self._tg_graph = g
        self._tg_graph.replay()
        return self._loss_buf

    def train(self, memory: RolloutBuffer):
        run, agent, eng, buf = self.run, self.agent, self.agent.engine, memory
        n, t_len, a = buf.num_envs, buf.horizon, buf.act_dim
        bs = run.training_config.batch_size
        epochs = int(run.training_config.epochs_per_iteration)
        exact = self.dp.world > 1 and self.dp.mode == "exact"
        # exact DP: ppo.py:97-106 over the GLOBAL buffer (single-process N*T and B)
        n_glob = self.dp.global_envs(n) if exact else n
        batches_per_epoch = int(t_len * n_glob / bs)
        if batches_per_epoch <= 0 or float(bs) != int(bs):
            # ppo.py:142: an epoch without a full minibatch divides by len([]) == 0
            raise ZeroDivisionError("division by zero")
        b = int(bs)
        dev = agent.device
        if self._rows is None or self._rows.numel() < b:
            self._rows = torch.empty(b, dtype=torch.int32, device=dev)
        if self._loss_buf is None or self._loss_buf.shape != (epochs, batches_per_epoch, 2):
            self._loss_buf = torch.empty(epochs, batches_per_epoch, 2, dtype=torch.float32,
                                         device=dev)
        ppo = run.ppo_config
        clip_lo = 1.0 - ppo.clip_epsilon
        clip_hi = 1.0 + ppo.clip_epsilon
        if exact:
            if self._count is None:
                self._count = torch.zeros(1, dtype=torch.int32, device=dev)
            if self._rng() != "torch":
                raise ValueError("exact data-parallel mode replays the reference RNG: rng='torch'")
        b_global = self.dp.loss_scale(b)
        inv_b = 1.0 / b_global
        inv_ba = 1.0 / (b_global * a)
        states = buf.states
        if self._scheduled_ok():
            out = self._train_scheduled(memory, b, epochs, batches_per_epoch, clip_lo, clip_hi,
                                        inv_b, inv_ba)
            if out is not None:
                if run.dynamic_config.current_episode < 2500:
                    for scheduler in agent.schedulers.values():
                        scheduler.step()
                return out
        staged = eng.fused
        # one 128 B record per stored row: the minibatch gathers read one line a row (staged
        # already when calculate_advantages ran the fused scan)
        if staged and not getattr(buf, "records_staged", False):
            eng.stage_records(states, buf.actions, buf.logp, buf.advantage, buf.value_target)
        buf.records_staged = False
        current = False  # bf16 weight images refreshed by the last optimizer step
        for epoch in range(epochs):
            if self._rng() == "torch":
                gen = None if exact else self._local_gen()
                perm = torch.randperm((n_glob if exact else n) * t_len,
                                      generator=gen).to(dev, non_blocking=True)
            for i in range(batches_per_epoch):
                count = None
                if exact:
                    torch.randn(b, a)  # ppo.py:110: agent.act draws a sample it never uses
                    E.perm_to_rows(perm, i * b, b, n_glob, t_len, self._rows,
                                   shard=self.dp.my_shard(n), count=self._count)
                    count = self._count
                elif self._rng() == "torch":
                    torch.randn(b, a, generator=gen)  # ppo.py:110
                    E.perm_to_rows(perm, i * b, b, n, t_len, self._rows)
                else:
                    E.feistel_rows(self._seed() + 7919 * self.dp.rank,
                                   self.iteration * epochs + epoch, i * b, b, n, t_len, self._rows)
                if staged:
                    eng.minibatch_grad_staged(self._rows, b, agent.flat_grad,
                                              self._loss_buf[epoch, i], clip_lo, clip_hi,
                                              ppo.entropy_eps, inv_b, inv_ba, count=count,
                                              weights_current=current)
                else:
                    eng.minibatch_grad(states, buf.actions, buf.logp, buf.advantage,
                                       buf.value_target, self._rows, b, agent.flat_grad,
                                       self._loss_buf[epoch, i], clip_lo, clip_hi,
                                       ppo.entropy_eps, inv_b, inv_ba, count=count)
                self.dp.allreduce_grad(agent.flat_grad)
                current = agent.step_both(pack=staged)
        if run.dynamic_config.current_episode < 2500:
            for scheduler in agent.schedulers.values():
                scheduler.step()
        return self._loss_buf

    def _finish_logging(self, loss_buf: torch.Tensor) -> None:
        if self.world > 1:
            # every rank's loss terms are already divided by the GLOBAL minibatch size
            # (DataParallel.loss_scale), so the SUM over ranks is the reference's per-minibatch
            # mean loss (ppo.py:139-153); one all-reduce per iteration, for logging only
            # (rank 0's entries alone carry the entropy bonus: DataParallel.attach)
            loss_buf = loss_buf.clone()
            self.dp.allreduce_log(loss_buf)
        losses = loss_buf.double().cpu()
        epoch_means = losses.mean(dim=1)
        actor_loss = float(epoch_means[:, 0].mean())
        critic_loss = float(epoch_means[:, 1].mean())
        self.last_losses = (actor_loss, critic_loss)

    # ---- base_algorithm.py:21-48: deterministic evaluation rollout ----------------------------
    @torch.no_grad()
    def test(self, visualize: bool = False, steps: int = 1000) -> float:
        """Algorithm.test: ``steps`` single-env steps with the mean action
        (agent.act(test_phase=True), flattened to (A,) as agent.py:35-38), reset on termination,
        window shift otherwise; returns sum(rewards) / len(rewards).

        Device-resident helpers (``test_step``) take the termination branch on the device and
        keep the f64 reward sum there, so the loop never synchronises the host until the final
        read; other helpers get the reference's host protocol (test_environment.step + branch).
        ``visualize`` is accepted for signature compatibility; rendering is out of scope."""
        helper, agent = self.environment_helper, self.agent
        agent.networks.eval()
        helper.reset_environment(test_phase=True)
        next_state = helper.get_state(test_phase=True)
        if hasattr(helper, "test_step"):
            reward_sum = torch.zeros(1, dtype=torch.float64, device=agent.device)
            for _ in range(steps):
                current_state = next_state  # get_state returns a fresh tensor (torch.clone, :29)
                action, _ = agent.act(current_state, return_dist=True, test_phase=True)
                helper.test_step(action.reshape(-1), reward_sum)
                next_state = helper.get_state(test_phase=True)
            mean_reward = float(reward_sum) / steps
        else:
            rewards = []
            ts = helper.test_timestep
            for _ in range(steps):
                current_state = torch.clone(next_state)
                action, _ = agent.act(current_state, return_dist=True, test_phase=True)
                last_obs, reward, ts.terminated, ts.truncated, _ = helper.test_environment.step(
                    action.reshape(-1).cpu().numpy())
                if ts.terminated:
                    helper.reset_environment(test_phase=True)
                else:
                    helper.shift_observations(test_phase=True, environment_index=-1)
                    ts.observation[:, -1] = torch.as_tensor(last_obs)
                rewards.append(reward)
                next_state = helper.get_state(test_phase=True)
            mean_reward = sum(rewards) / len(rewards)
        agent.networks.train()
        return mean_reward

    # ---- ppo.py:156-159, base_algorithm.py:53-58 ----------------------------------------------
    def _iterate(self):
        memory = self.rollout()
        self.calculate_advantages(memory)
        loss_buf = self.train(memory)
        self.iteration += 1
        return memory, loss_buf

    def iterate(self, verbose: bool = True):
        t0 = time.perf_counter()
        memory, loss_buf = self._iterate()
        self._finish_logging(loss_buf)
        self.last_mean_reward = float(memory.reward.mean())
        run = self.run
        if verbose:
            ep = run.dynamic_config.current_episode
            self.log(f"[iteration {ep}] total episode reward: {self.last_mean_reward}")
            self.log(f"Actor Loss: {self.last_losses[0]} Critic Loss: {self.last_losses[1]} "
                     f"Epoch Loss: {self.last_losses[0] + self.last_losses[1]}")
            self.log(f"iterate took {time.perf_counter() - t0:.4f} s")
        run.dynamic_config.next_episode()
        return memory
