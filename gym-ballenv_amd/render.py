"""Optional host-side render of env 0 (the reference renders with a pyglet
viewer, ballenv_env.py:357-386; pygame is optional and absent here).

``rgb_array`` rasterises env 0's agent (radius_agent), goal (10x10 square) and
obstacles (radius_obstacle; static red, dynamic green, as ballenv_env.py:295-314)
into an (H, W, 3) uint8 array with y up, like the reference's viewer.
"""
from __future__ import annotations

import numpy as np


def _disk(img, cx, cy, r, color):
    H, W, _ = img.shape
    y0, y1 = max(int(cy - r), 0), min(int(cy + r) + 1, H)
    x0, x1 = max(int(cx - r), 0), min(int(cx + r) + 1, W)
    if y0 >= y1 or x0 >= x1:
        return
    yy, xx = np.mgrid[y0:y1, x0:x1]
    m = (xx - cx) ** 2 + (yy - cy) ** 2 <= r * r
    img[y0:y1, x0:x1][m] = color


def rgb_array(env, index: int = 0) -> np.ndarray:
    cfg = env.cfg
    H, W = cfg.screen_height + 1, cfg.screen_width + 1
    img = np.full((H, W, 3), 255, np.uint8)
    ag = env.agent[index].tolist()
    go = env.goal[index].tolist()
    for p in env.static_obs[:cfg.num_static, index].tolist():
        _disk(img, p[0], p[1], cfg.radius_obstacle, (100, 0, 0))
    for p in env.dyn_obs[:cfg.num_dynamic, index].tolist():
        _disk(img, p[0], p[1], cfg.radius_obstacle, (0, 100, 0))
    gx, gy = go
    img[max(gy - 5, 0):max(gy + 6, 0), max(gx - 5, 0):max(gx + 6, 0)] = (0, 0, 0)
    _disk(img, ag[0], ag[1], cfg.radius_agent, (0, 0, 255))
    return img[::-1].copy()  # y up


def render_env0(env, mode: str = "rgb_array"):
    img = rgb_array(env, 0)
    if mode == "rgb_array":
        return img
    if mode == "human":
        try:
            import pygame  # noqa: F401
        except ImportError as e:
            raise RuntimeError("render(mode='human') needs pygame; use mode='rgb_array'") from e
        import pygame
        if not pygame.display.get_init():
            pygame.display.init()
        surf = pygame.display.set_mode((img.shape[1], img.shape[0]))
        pygame.surfarray.blit_array(surf, img.swapaxes(0, 1))
        pygame.display.flip()
        return None
    raise ValueError(f"unknown render mode {mode!r}")
