"""BatchedBoard: N ``ballenv_pygame.createBoard`` worlds on the GPU.

The reference's other physics profile (ballenv_pygame.py:314-706): a 100x100 field with
f64 positions (ranf spawns), static obstacles, 4 keyboard actions (actionArray :352-353)
or float mouse moves, reward -1 on a hit / +1 at the goal / (old-cur)/total otherwise
(calc_reward :680-706), and after every step the 20 IRL features of
``featureExtractor.featureExtractor`` (featureExtractor.py:247-265), which is what the IRL
drivers read as ``sensor_readings``.  Every step / reset / observe is one launch of
``csrc/board.hip`` through the C ABI (``be_board_*`` in include/ballenv.h); there is no
CPU fallback.

    board = BatchedBoard(65536, num_static=6)
    feats = board.reset()                              # (N, 20) f32 sensor_readings
    feats, reward, done, info = board.step(actions)    # actions: (N,) indices into actionArray
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import _abi

ACTIONS = [(0, -1), (1, 0), (0, 1), (-1, 0)]


class BatchedBoard:
    STATE_KEYS = ("agent", "goal", "dist", "total_dist", "ep_return", "ep_len", "episode", "static_obs")

    def __init__(self, num_envs: int, num_static: int = 0, device="cuda", seed: int = 0xB0A2D, env_offset: int = 0,
                 autoreset: bool = False, time_limit: int = 0, **overrides):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("BatchedBoard runs on a GPU device only (no CPU fallback)")
        self.num_envs, self.num_static = int(num_envs), int(num_static)
        self._lib = _abi.lib()
        c = _abi.BeBoardConfig()
        _abi.board_check(self._lib.be_board_config_default(C.byref(c), self.num_envs, self.num_static))
        c.seed, c.env_offset = int(seed) & (2**64 - 1), int(env_offset)
        c.autoreset, c.time_limit = int(bool(autoreset)), int(time_limit)
        for k, v in overrides.items():
            if k == "actions":
                c.num_actions = len(v)
                for a, (dx, dy) in enumerate(v):
                    c.actions[a][0], c.actions[a][1] = float(dx), float(dy)
            else:
                setattr(c, k, v)
        self.cfg = c
        h = C.c_void_p()
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        _abi.board_check(self._lib.be_board_create(C.byref(c), dev, C.byref(h)))
        self._h = h
        N, d = self.num_envs, self.device
        z = lambda *shape, dt: torch.zeros(*shape, dtype=dt, device=d)  # noqa: E731
        self.agent, self.goal = z(N, 2, dt=torch.float64), z(N, 2, dt=torch.float64)
        self.dist, self.total_dist, self.ep_return = z(N, dt=torch.float64), z(N, dt=torch.float64), z(N, dt=torch.float64)
        self.ep_len, self.episode = z(N, dt=torch.int32), z(N, dt=torch.int32)
        self.static_obs = z(max(self.num_static, 1), N, 2, dt=torch.int16)
        self.features = z(N, _abi.BOARD_FEATURES, dt=torch.float32)
        self.reward, self.done, self.truncated = z(N, dt=torch.float64), z(N, dt=torch.bool), z(N, dt=torch.bool)
        self._st = _abi.BeBoardState(*[getattr(self, k).data_ptr() for k in self.STATE_KEYS])
        self._out = _abi.BeBoardOut(self.features.data_ptr(), self.reward.data_ptr(), self.done.data_ptr(),
                                    self.truncated.data_ptr())

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def total_reward_accumulated(self) -> torch.Tensor:
        return self.ep_return

    @property
    def sensor_readings(self) -> torch.Tensor:
        return self.features

    def reset(self, mask: Optional[torch.Tensor] = None, reset_tape: Optional[torch.Tensor] = None) -> torch.Tensor:
        """createBoard.reset for all envs (or mask != 0); returns the (N, 20) features.
        reset_tape: (L, N) f64 -- the reference's ranf / randint values in call order."""
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        t, L = None, 0
        if reset_tape is not None:
            t = reset_tape.to(device=self.device, dtype=torch.float64).contiguous()
            L = t.shape[0]
        _abi.board_check(self._lib.be_board_reset(self._h, C.byref(self._st), None if m is None else m.data_ptr(),
                                                  None if t is None else t.data_ptr(), L, C.byref(self._out),
                                                  self._stream()), self._h)
        self._keep = (m, t)
        return self.features

    def step(self, actions: Optional[torch.Tensor] = None, deltas: Optional[torch.Tensor] = None):
        """createBoard.step + featureExtractor: actions (N,) indices into actionArray, or
        deltas (N, 2) f64 moves.  Returns (features, reward, done, info)."""
        a = d = None
        if actions is not None:
            a = actions.to(device=self.device, dtype=torch.uint8).contiguous()
        elif deltas is not None:
            d = deltas.to(device=self.device, dtype=torch.float64).contiguous()
        else:
            raise ValueError("step needs actions or deltas")
        _abi.board_check(self._lib.be_board_step(self._h, C.byref(self._st), None if a is None else a.data_ptr(),
                                                 None if d is None else d.data_ptr(), C.byref(self._out),
                                                 self._stream()), self._h)
        self._keep = (a, d)
        return self.features, self.reward, self.done, {"truncated": self.truncated}

    def rollout(self, actions: Optional[torch.Tensor] = None, deltas: Optional[torch.Tensor] = None):
        """K steps in one launch (be_board_rollout): actions (K, N) indices or deltas (K, N, 2).
        Returns per-step (features (K, N, 20), reward (K, N), done (K, N), info{truncated}),
        exactly what K step() calls return, stacked.  The buffers are reused by the next
        rollout of the same K."""
        a = d = None
        if actions is not None:
            a = actions.to(device=self.device, dtype=torch.uint8).contiguous()
            K = a.shape[0]
            if a.dim() != 2 or a.shape[1] != self.num_envs:
                raise ValueError(f"actions must be (K, {self.num_envs})")
        elif deltas is not None:
            d = deltas.to(device=self.device, dtype=torch.float64).contiguous()
            K = d.shape[0]
            if d.dim() != 3 or d.shape[1:] != (self.num_envs, 2):
                raise ValueError(f"deltas must be (K, {self.num_envs}, 2)")
        else:
            raise ValueError("rollout needs actions or deltas")
        N = self.num_envs
        buf = getattr(self, "_ro_buf", None)
        if buf is None or buf[0].shape[0] != K:
            z = lambda *shape, dt: torch.zeros(*shape, dtype=dt, device=self.device)  # noqa: E731
            buf = (z(K, N, _abi.BOARD_FEATURES, dt=torch.float32), z(K, N, dt=torch.float64), z(K, N, dt=torch.bool),
                   z(K, N, dt=torch.bool))
            self._ro_buf = buf
        f, r, dn, tr = buf
        out = _abi.BeBoardOut(f.data_ptr(), r.data_ptr(), dn.data_ptr(), tr.data_ptr())
        _abi.board_check(self._lib.be_board_rollout(self._h, C.byref(self._st), None if a is None else a.data_ptr(),
                                                    None if d is None else d.data_ptr(), int(K), C.byref(out),
                                                    self._stream()), self._h)
        self._keep = (a, d)
        return f, r, dn, {"truncated": tr}

    def observe(self) -> torch.Tensor:
        _abi.board_check(self._lib.be_board_observe(self._h, C.byref(self._st), C.byref(self._out), self._stream()),
                         self._h)
        return self.features

    def status(self) -> int:
        v = C.c_int32()
        _abi.board_check(self._lib.be_board_status(self._h, C.byref(v), self._stream()), self._h)
        if v.value:
            bits = [txt for bit, txt in _abi.STATUS_BITS.items() if v.value & bit]
            raise _abi.BallEnvError("device status: " + "; ".join(bits))
        return 0

    def pool_bytes(self) -> int:
        """Bytes of the autoreset pool (be_board_pool_bytes; 0: every reset drawn inline)."""
        f = getattr(self._lib, "be_board_pool_bytes", None)
        return int(f(self._h)) if f is not None and f.restype is not None else 0

    def state_dict(self) -> dict:
        return {k: getattr(self, k).clone() for k in self.STATE_KEYS}

    def load_state_dict(self, d: dict) -> None:
        for k in self.STATE_KEYS:
            dst = getattr(self, k)
            src = d[k]
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f"state '{k}': shape {tuple(src.shape)} != {tuple(dst.shape)}")
            dst.copy_(src.to(device=self.device, dtype=dst.dtype))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            torch.cuda.synchronize(self.device)
            self._lib.be_board_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
