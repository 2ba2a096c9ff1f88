"""BatchedBallEnv: N independent BallEnvs as a struct-of-arrays on one GPU.

Host side of the drop-in boundary.  The per-env state lives in caller-owned
PyTorch tensors (env index = unit stride); every reset/step/observe is one
asynchronous launch of the HIP kernels in libballenv.so on the current torch
stream, through the C ABI of include/ballenv.h.  Nothing here computes physics
or observations on the CPU, and there is no fallback path.

Reference surface this mirrors (gym.Env protocol used by examples/ball_cnn_ac3.py):
* ``reset()``  <- BallEnv.reset        gym_ballenv/envs/ballenv_env.py:113-167 (+ prep_state4)
* ``step(a)``  <- BallEnv.step         ballenv_env.py:232-289, then prep_state4
                  (examples/ball_cnn_ac3.py:384-412), under the TimeLimit(1000) of
                  gym_ballenv/__init__.py:4-11
* ``customize_environment(args)``      ballenv_env.py:87-109
* ``total_reward_accumulated``         ballenv_env.py:66,129,280 (here an (N,) f64 view)
* ``observation_space/action_space``   the shapes step() really returns / accepts
                  (the reference declares Box(2)/Discrete(4), ballenv_env.py:57-58, Q11)
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Optional

import torch

from . import _abi
from .config import EnvConfig
from .spaces import Box, Discrete


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class BatchedBallEnv:
    """``num_envs`` BallEnvs stepped by one kernel launch per call.

    Returned tensors (obs, reward, done, info entries) are views of internal
    buffers that the next call overwrites; ``.clone()`` what you keep.
    """

    # SoA state tensors, in be_state field order (include/ballenv.h)
    STATE_KEYS = ("agent", "goal", "prev_dist", "total_dist", "ep_return", "ep_len", "episode", "static_obs",
                  "dyn_obs", "dyn_goal")

    def __init__(self, num_envs: int, window: int = 10, config: Optional[EnvConfig] = None,
                 device="cuda", seed: int = 0xBA11, env_offset: int = 0, obs_f32: bool = False,
                 track_stats: bool = True, terminal_obs: bool = False):
        self.num_envs, self.window = int(num_envs), int(window)
        self.cfg = config if config is not None else EnvConfig()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("BatchedBallEnv runs on a GPU device only (no CPU fallback)")
        self.seed, self.env_offset = int(seed), int(env_offset)
        self.obs_dim = 4 + self.window * self.window
        self._want_f32, self._want_terminal, self._track_stats = obs_f32, terminal_obs, track_stats
        self._lib = _abi.lib()
        self._ctx = None
        self._alloc()
        self._create_ctx()

    # ------------------------------------------------------------------ setup
    def _alloc(self):
        N, dev, cfg = self.num_envs, self.device, self.cfg
        z = lambda *shape, dt: torch.zeros(*shape, dtype=dt, device=dev)  # noqa: E731
        self.agent = z(N, 2, dt=torch.int16)
        self.goal = z(N, 2, dt=torch.int16)
        self.prev_dist = z(N, dt=torch.float64)
        self.total_dist = z(N, dt=torch.float64)
        self.ep_return = z(N, dt=torch.float64)
        self.ep_len = z(N, dt=torch.int32)
        self.episode = z(N, dt=torch.int32)      # uint32 on the device side
        self.static_obs = z(max(cfg.num_static, 1), N, 2, dt=torch.int16)
        self.dyn_obs = z(max(cfg.num_dynamic, 1), N, 2, dt=torch.int16)
        self.dyn_goal = z(max(cfg.num_dynamic, 1), N, dt=torch.uint8)
        F = self.obs_dim
        self.obs = z(N, F, dt=torch.uint8)
        self.obs_f32 = z(N, F, dt=torch.float32) if self._want_f32 else None
        self.reward = z(N, dt=torch.float64)
        self.done = z(N, dt=torch.bool)
        self.truncated = z(N, dt=torch.bool)
        self.final_return = z(N, dt=torch.float64)
        self.final_len = z(N, dt=torch.int32)
        self.terminal_obs = z(N, F, dt=torch.uint8) if self._want_terminal else None
        self.stats_buf = z(_abi.stats_slots(cfg.to_abi(N, self.window)), 8, dt=torch.float64)
        self.clear_stats()
        self._st = _abi.BeState(*[getattr(self, k).data_ptr() for k in self.STATE_KEYS])
        self._out = _abi.BeOut(self.obs.data_ptr(), _ptr(self.obs_f32), self.reward.data_ptr(),
                               self.done.data_ptr(), self.truncated.data_ptr(), _ptr(self.terminal_obs),
                               self.final_return.data_ptr(), self.final_len.data_ptr(),
                               self.stats_buf.data_ptr() if self._track_stats else None)
        # per-call constants of step(): the ctypes references and the info dict (its values are the
        # same buffers every step), built once instead of on every call
        self._st_ref, self._out_ref = C.byref(self._st), C.byref(self._out)
        self._info = {"truncated": self.truncated, "final_return": self.final_return, "final_len": self.final_len}
        if self.terminal_obs is not None:
            self._info["terminal_obs"] = self.terminal_obs
        self._obs_ret = self.obs_f32 if self._want_f32 else self.obs
        self._a_ok = None       # the last actions tensor that passed step()'s checks as it was

    def _create_ctx(self):
        if self._ctx is not None:
            self._lib.be_destroy(self._ctx)
            self._ctx = None
        self._abi_cfg = self.cfg.to_abi(self.num_envs, self.window, self.env_offset, self.seed)
        msg = _abi.config_check(self._abi_cfg)
        if msg:
            raise ValueError(f"invalid BallEnv config: {msg}")
        ctx = C.c_void_p()
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        _abi.check(self._lib.be_create(C.byref(self._abi_cfg), dev, C.byref(ctx)))
        self._ctx = ctx
        self._dev_index = dev
        # the raw current-stream getter saves host time per step(); it is private torch API, so a
        # torch without it falls back to the public Stream object (same handle, a little slower)
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            self._stream = lambda: C.c_void_p(raw(dev))
        else:
            self._stream = lambda: C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def _stream(self):
        """The caller's current stream on this env's device (raw handle; replaced per instance in
        _create_ctx by the fastest getter this torch has)."""
        return C.c_void_p(torch.cuda.current_stream(self._dev_index).cuda_stream)

    # ------------------------------------------------------------------ gym surface
    @property
    def observation_space(self) -> Box:
        return Box(0.0, 1.0, (self.obs_dim,))

    @property
    def action_space(self) -> Discrete:
        return Discrete(len(self.cfg.actions))

    @property
    def total_reward_accumulated(self) -> torch.Tensor:
        return self.ep_return

    def customize_environment(self, args) -> None:
        """ballenv_env.py:87-109: reconfigure from ball_cnn_ac3.py-style argparse args."""
        self.cfg = EnvConfig.from_args(args, self.cfg)
        self._alloc()
        self._create_ctx()

    def reset(self, mask: Optional[torch.Tensor] = None, reset_tape: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reset all envs (or those with mask != 0); returns the obs of every env.

        ``reset_tape``: optional (L, N) int16 randint values in the reference's
        call order (parity mode); otherwise Philox draws keyed by global env id.
        """
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            self._check_shape(m, (self.num_envs,), "mask")
        L = 0
        if reset_tape is not None:
            reset_tape = reset_tape.to(device=self.device, dtype=torch.int16).contiguous()
            if reset_tape.dim() != 2 or reset_tape.shape[1] != self.num_envs:
                raise ValueError("reset_tape must be (L, num_envs) int16")
            L = reset_tape.shape[0]
        _abi.check(self._lib.be_reset(self._ctx, C.byref(self._st), _ptr(m), _ptr(reset_tape), L,
                                      C.byref(self._out), self._stream()), self._ctx)
        self._keep = (m, reset_tape)
        return self.obs_f32 if self._want_f32 else self.obs

    def step(self, actions: Optional[torch.Tensor] = None, deltas: Optional[torch.Tensor] = None,
             draw_tape: Optional[torch.Tensor] = None, copy: bool = False):
        """One step of every env.

        actions: (N,) integer indices into ``cfg.actions`` (the move_list of
        ball_cnn_ac3.py:530); or deltas: (N, 2) raw (dx, dy) as BallEnv.step takes;
        neither: uniformly sampled actions (Philox, keyed by global env id).
        draw_tape: (Nd, 2, N) int16 obstacle-move randint values (parity mode).
        Returns (obs, reward f64, done bool, info).

        Return semantics: with ``copy=False`` (the default, no allocation per step) obs, reward,
        done and the info tensors are the env's output buffers, overwritten by the NEXT step --
        a caller that keeps per-step outputs (``rewards.append(reward)``, ball_cnn_ac3.py:610)
        must ``.clone()`` them.  ``copy=True`` returns fresh tensors each call, as
        BallEnv.step returns a fresh np.array and float (ballenv_env.py:289).
        """
        if copy:
            obs, reward, done, info = self.step(actions, deltas, draw_tape)
            return obs.clone(), reward.clone(), done.clone(), {k: v.clone() for k, v in info.items()}
        if actions is not None and deltas is None and draw_tape is None:
            # the common call (ball_cnn_ac3.py:588 for every env): the same (N,) u8 action buffer
            # each step skips the re-checks -- one ctypes call, the info dict prebuilt (the host
            # cost per call is bench.py's eager_step leg)
            if (actions is not self._a_ok or actions.dtype != torch.uint8 or actions.shape != self._a_shape
                    or actions.data_ptr() != self._a_ptr):
                a = actions if actions.dtype == torch.uint8 else actions.to(torch.uint8)
                if a.device != self.device:
                    a = a.to(self.device)
                a = a.contiguous()
                self._check_shape(a, (self.num_envs,), "actions")
                if a is not actions:          # a converted copy: keep it alive for the async launch
                    self._keep = (a,)
                    self._a_ok = None
                else:
                    self._a_ok, self._a_shape, self._a_ptr = a, a.shape, a.data_ptr()
                ptr = a.data_ptr()
            else:
                ptr = self._a_ptr
            rc = self._lib.be_step(self._ctx, self._st_ref, ptr, None, None, self._out_ref, self._stream())
            if rc:
                _abi.check(rc, self._ctx)
            return self._obs_ret, self.reward, self.done, self._info
        a = d = t = None
        if actions is not None:
            a = actions if actions.dtype == torch.uint8 else actions.to(torch.uint8)
            if a.device != self.device:
                a = a.to(self.device)
            a = a.contiguous()
            self._check_shape(a, (self.num_envs,), "actions")
        elif deltas is not None:
            d = deltas.to(device=self.device, dtype=torch.int16).contiguous()
            self._check_shape(d, (self.num_envs, 2), "deltas")
        if draw_tape is not None:
            t = draw_tape.to(device=self.device, dtype=torch.int16).contiguous()
            if self.cfg.num_dynamic:
                self._check_shape(t, (self.cfg.num_dynamic, 2, self.num_envs), "draw_tape")
        _abi.check(self._lib.be_step(self._ctx, C.byref(self._st), _ptr(a), _ptr(d), _ptr(t),
                                     C.byref(self._out), self._stream()), self._ctx)
        self._keep = (a, d, t)
        return self._obs_ret, self.reward, self.done, self._info

    def rollout(self, actions: torch.Tensor):
        """``K = actions.shape[0]`` consecutive steps in one launch (be_rollout).

        actions: (K, N) integer indices into ``cfg.actions``.  Returns per-step
        ``(obs (K, N, F) u8, reward (K, N) f64, done (K, N) bool, info)`` with info
        ``truncated`` / ``final_return`` / ``final_len`` (K, N) -- exactly what K calls of
        :meth:`step` return, stacked (the reference's per-step loop of
        examples/ball_cnn_ac3.py:573-600, for every env).  The state advances by K steps.
        With ``terminal_obs=True`` info also holds ``terminal_obs`` (K, N, F), written for
        the rows of envs that reset on that step.  u8 obs only; the buffers are reused by the
        next rollout of the same K.
        """
        if self._want_f32:
            raise ValueError("rollout() returns u8 obs only (build the env without obs_f32)")
        a = actions if actions.dtype == torch.uint8 else actions.to(torch.uint8)
        if a.device != self.device:
            a = a.to(self.device)
        a = a.contiguous()
        if a.dim() != 2 or a.shape[1] != self.num_envs:
            raise ValueError(f"actions must be (K, {self.num_envs}), got {tuple(a.shape)}")
        K, N, F = a.shape[0], self.num_envs, self.obs_dim
        buf = getattr(self, "_ro_buf", None)
        if buf is None or buf[0].shape[0] != K:
            z = lambda *shape, dt: torch.zeros(*shape, dtype=dt, device=self.device)  # noqa: E731
            buf = (z(K, N, F, dt=torch.uint8), z(K, N, dt=torch.float64), z(K, N, dt=torch.bool),
                   z(K, N, dt=torch.bool), z(K, N, dt=torch.float64), z(K, N, dt=torch.int32),
                   z(K, N, F, dt=torch.uint8) if self._want_terminal else None)
            self._ro_buf = buf
        obs, reward, done, trunc, fret, flen, term = buf
        out = _abi.BeOut(obs.data_ptr(), None, reward.data_ptr(), done.data_ptr(), trunc.data_ptr(), _ptr(term),
                         fret.data_ptr(), flen.data_ptr(), self.stats_buf.data_ptr() if self._track_stats else None)
        _abi.check(self._lib.be_rollout(self._ctx, C.byref(self._st), a.data_ptr(), int(K), C.byref(out),
                                        self._stream()), self._ctx)
        self._keep = (a,)
        info = {"truncated": trunc, "final_return": fret, "final_len": flen}
        if term is not None:
            info["terminal_obs"] = term
        return obs, reward, done, info

    def step_n(self, actions: torch.Tensor):
        """``K = actions.shape[0]`` consecutive :meth:`step` calls (caller actions), queued by one
        library call (be_step_n: one kernel launch per step from a C loop).  Returns what the
        last :meth:`step` would: ``(obs, reward, done, info)`` of step K."""
        a = actions if actions.dtype == torch.uint8 else actions.to(torch.uint8)
        if a.device != self.device:
            a = a.to(self.device)
        a = a.contiguous()
        if a.dim() != 2 or a.shape[1] != self.num_envs:
            raise ValueError(f"actions must be (K, {self.num_envs}), got {tuple(a.shape)}")
        _abi.check(self._lib.be_step_n(self._ctx, C.byref(self._st), a.data_ptr(), int(a.shape[0]),
                                       C.byref(self._out), self._stream()), self._ctx)
        self._keep = (a,)
        info = {"truncated": self.truncated, "final_return": self.final_return, "final_len": self.final_len}
        if self.terminal_obs is not None:
            info["terminal_obs"] = self.terminal_obs
        return (self.obs_f32 if self._want_f32 else self.obs), self.reward, self.done, info

    def observe(self) -> torch.Tensor:
        """prep_state4 of the current state (no state change)."""
        _abi.check(self._lib.be_observe(self._ctx, C.byref(self._st), C.byref(self._out), self._stream()), self._ctx)
        return self.obs_f32 if self._want_f32 else self.obs

    def observe_blocks(self, f32: bool = False) -> torch.Tensor:
        """prep_state2 of examples/ball_env_reinforce.py:130-172 for the current state:
        (N, 29) block counts (u8, or f32 with ``f32=True``) -- the input of the
        REINFORCE / supervised policies (29 = 4 quadrant + 5x5 blocks)."""
        dt = torch.float32 if f32 else torch.uint8
        out = torch.empty(self.num_envs, 29, dtype=dt, device=self.device)
        u8, f = (None, out.data_ptr()) if f32 else (out.data_ptr(), None)
        _abi.check(self._lib.be_observe_blocks(self._ctx, C.byref(self._st), u8, f, self._stream()), self._ctx)
        return out

    def window_only(self) -> torch.Tensor:
        """(N, W*W) view of the window part of the obs: prep_state4 as the potential-field
        planners define it, without the quadrant (examples/potential_fields_modified.py:66-93)."""
        return (self.obs_f32 if self._want_f32 else self.obs)[:, 4:]

    def sample_actions(self, steps: int, seed: int = 0xBA11) -> torch.Tensor:
        """(steps, N) u8 uniform action indices from Philox(seed; global env id, t)."""
        out = torch.empty(steps, self.num_envs, dtype=torch.uint8, device=self.device)
        _abi.check(self._lib.be_sample_actions(self._ctx, out.data_ptr(), int(steps), int(seed) & (2**64 - 1),
                                               self._stream()), self._ctx)
        return out

    def kernel_name(self, entry: str = "step") -> Optional[str]:
        """Name of the kernel an entry point launches for this env (rocprofv3's kernel name
        without namespace / arguments): entry in step (caller actions), step_sampled,
        rollout (None when be_rollout falls back to looping be_step), reset, observe."""
        ids = {"step": 0, "step_sampled": 1, "rollout": 2, "reset": 3, "observe": 4}
        r = self._lib.be_kernel_name(self._ctx, ids[entry])
        return r.decode() if r else None

    # ------------------------------------------------------------------ the autoreset pool
    # (include/ballenv.h: precomputed next-episode resets the fixed-shape step kernels copy on done;
    # results are bit-identical with or without it -- these calls change timing only)
    def pool_bytes(self) -> int:
        """Device bytes of this env's autoreset pool (0: its step kernel draws every reset inline;
        also 0 for a BALLENV_LIB diagnostics build that predates the pool)."""
        fn = getattr(self._lib, "be_pool_bytes", None)
        return int(fn(self._ctx)) if fn is not None else 0

    def pool_fill(self) -> None:
        """Draw every env's stale entries now (be_pool_fill), on the current stream."""
        _abi.check(self._lib.be_pool_fill(self._ctx, C.byref(self._st), self._stream()), self._ctx)

    def pool_invalidate(self) -> None:
        """Mark every entry unwritten: resets are drawn inline until the next fill."""
        _abi.check(self._lib.be_pool_invalidate(self._ctx, self._stream()), self._ctx)

    def pool_period(self) -> int:
        """Step launches per queued fill (0: fills only at reset / load_state / pool_fill)."""
        return int(self._lib.be_pool_period(self._ctx))

    def pool_set_period(self, period: int) -> None:
        """be_step queues a fill every ``period`` steps (0: only reset / load_state / pool_fill)."""
        _abi.check(self._lib.be_pool_set_period(self._ctx, int(period)), self._ctx)

    def pool_entry(self, env: int, slot: int, write=None):
        """Test hook: (words u32 (6 + Ns + Nd,), f64 (2,)) of env's entry in slot (episode & 1), or
        overwrite it with ``write = (words, f64)``.  Synchronises the device."""
        nw = 6 + self.cfg.num_static + self.cfg.num_dynamic
        w, d = (C.c_uint32 * nw)(), (C.c_double * 2)()
        if write is not None:
            for k, v in enumerate(write[0]):
                w[k] = int(v) & 0xFFFFFFFF
            d[0], d[1] = float(write[1][0]), float(write[1][1])
        _abi.check(self._lib.be_pool_entry(self._ctx, int(env), int(slot), w, d, 1 if write is not None else 0),
                   self._ctx)
        return list(w), list(d)

    # ------------------------------------------------------------------ bookkeeping
    def status(self) -> int:
        """Synchronise and read (then clear) the device status word; raises on error bits."""
        v = C.c_int32()
        _abi.check(self._lib.be_status(self._ctx, C.byref(v), self._stream()), self._ctx)
        if v.value:
            bits = [txt for bit, txt in _abi.STATUS_BITS.items() if v.value & bit]
            raise _abi.BallEnvError("device status: " + "; ".join(bits))
        return 0

    def clear_stats(self) -> None:
        self.stats_buf.zero_()
        self.stats_buf[:, 4] = math.inf
        self.stats_buf[:, 5] = -math.inf

    def stats_record(self) -> torch.Tensor:
        """(8,) f64 on the device: the per-block slots reduced (sums add, min/max reduce)."""
        b = self.stats_buf
        r = b.sum(0)
        r[4] = b[:, 4].min()
        r[5] = b[:, 5].max()
        return r

    def episode_stats(self) -> dict:
        s = self.stats_record().cpu().tolist()
        n = s[0]
        return {"episodes": int(n), "mean_return": s[1] / n if n else float("nan"),
                "sum_return": s[1], "sum_return_sq": s[2], "mean_length": s[3] / n if n else float("nan"),
                "min_return": s[4], "max_return": s[5]}


    def state_dict(self) -> dict:
        """SoA snapshot (env-state checkpoint; SURVEY §5 'Checkpoint / resume')."""
        return {k: getattr(self, k).clone() for k in self.STATE_KEYS}

    def load_state_dict(self, d: dict) -> None:
        for k in self.STATE_KEYS:
            src = d[k]
            dst = getattr(self, k)
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f"state '{k}': shape {tuple(src.shape)} != {tuple(dst.shape)}")
            if hasattr(torch, "uint32") and src.dtype == torch.uint32:
                src = src.view(torch.int32)
            dst.copy_(src.to(device=self.device, dtype=dst.dtype))

    def save_state(self, device=None) -> torch.Tensor:
        """be_save_state: every env's state packed into one u8 blob (include/ballenv.h layout:
        64-byte header, then the be_state arrays), on this env's device or ``device`` ("cpu":
        pinned host memory).  A device blob fills asynchronously on the current stream; a host
        blob is complete when this returns.  load_state() checks the blob's length and header,
        and returns only after a host blob has been read."""
        n = int(self._lib.be_state_blob_bytes(C.byref(self._abi_cfg)))
        dev = self.device if device is None else torch.device(device)
        blob = torch.empty(n, dtype=torch.uint8, device=dev, pin_memory=dev.type == "cpu")
        _abi.check(self._lib.be_save_state(self._ctx, C.byref(self._st), blob.data_ptr(), self._stream()), self._ctx)
        if dev.type == "cpu":      # a host blob is complete on return (ready for torch.save)
            torch.cuda.current_stream(self.device).synchronize()
        return blob

    def load_state(self, blob: torch.Tensor) -> None:
        """be_load_state: restore every env's state from a save_state() blob (header checked)."""
        if blob.dtype != torch.uint8 or not blob.is_contiguous():
            raise ValueError("blob must be a contiguous uint8 tensor from save_state()")
        n = int(self._lib.be_state_blob_bytes(C.byref(self._abi_cfg)))
        if blob.numel() < n:
            raise ValueError(f"blob holds {blob.numel()} bytes, this env's state needs {n} (truncated blob?)")
        host = blob.device.type == "cpu"
        if host and not blob.is_pinned():
            blob = blob.pin_memory()
        _abi.check(self._lib.be_load_state(self._ctx, C.byref(self._st), blob.data_ptr(), self._stream()), self._ctx)
        if host:                   # the copies have read the host blob before it can be dropped or reused
            torch.cuda.current_stream(self.device).synchronize()

    def close(self) -> None:
        if self._ctx is not None:
            torch.cuda.synchronize(self.device)
            self._lib.be_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _check_shape(t: torch.Tensor, shape, name: str) -> None:
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
