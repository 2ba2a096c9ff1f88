"""Optional host-side render of env 0 (the reference's BallEnv.render, ballenv_env.py:357-386,
drawn by gym's pyglet ``rendering.Viewer``; pyglet and pygame are absent here, so the viewer
itself is not run -- render parity is unpinned, the geometry below follows the reference's code).

What the reference's viewer draws, in its order (geoms are drawn in the order they were added):

* the controlled agent: ``make_circle(radius_ctrl_person)``, default colour black (:365-367);
* the goal: ``FilledPolygon([(5,5),(5,-5),(-5,5),(-5,-5)])``, black (:369-372).  That vertex
  order is a self-intersecting quad; GL_POLYGON fills it as the fan of triangles (v0,v1,v2),
  (v0,v2,v3), i.e. the 10x10 square minus its lower quarter below both diagonals;
* the obstacles, statics then dynamics (obstacle_list order): ``make_circle(radius_rand_person)``
  with ``set_color(100,0,0)`` / ``set_color(0,100,0)`` (:295-309) -- gym's colours are floats in
  [0, 1], so GL clamps them to pure red / pure green.

The window is screen_width x screen_height on a white background with y up; ``rgb_array``
returns it top row first, as ``viewer.render(return_rgb_array=True)`` does.  ``human`` shows the
same image through pygame when it is installed.
"""
from __future__ import annotations

import numpy as np

BLACK, RED, GREEN, WHITE = (0, 0, 0), (255, 0, 0), (0, 255, 0), (255, 255, 255)
GOAL_POLY = ((5, 5), (5, -5), (-5, 5), (-5, -5))   # ballenv_env.py:369


def _disk(img, cx, cy, r, color):
    """Pixels whose centre (x + 0.5, y + 0.5) lies within r of (cx, cy)."""
    H, W, _ = img.shape
    y0, y1 = max(int(np.floor(cy - r)), 0), min(int(np.ceil(cy + r)) + 1, H)
    x0, x1 = max(int(np.floor(cx - r)), 0), min(int(np.ceil(cx + r)) + 1, W)
    if y0 >= y1 or x0 >= x1:
        return
    yy, xx = np.mgrid[y0:y1, x0:x1]
    m = (xx + 0.5 - cx) ** 2 + (yy + 0.5 - cy) ** 2 <= r * r
    img[y0:y1, x0:x1][m] = color


def _triangle(img, pts, color):
    """Fill a triangle (pixel-centre test, either winding)."""
    H, W, _ = img.shape
    (ax, ay), (bx, by), (cx, cy) = pts
    x0, x1 = max(int(np.floor(min(ax, bx, cx))), 0), min(int(np.ceil(max(ax, bx, cx))) + 1, W)
    y0, y1 = max(int(np.floor(min(ay, by, cy))), 0), min(int(np.ceil(max(ay, by, cy))) + 1, H)
    if y0 >= y1 or x0 >= x1:
        return
    yy, xx = np.mgrid[y0:y1, x0:x1]
    px, py = xx + 0.5, yy + 0.5

    def edge(x0_, y0_, x1_, y1_):
        return (x1_ - x0_) * (py - y0_) - (y1_ - y0_) * (px - x0_)

    e0, e1, e2 = edge(ax, ay, bx, by), edge(bx, by, cx, cy), edge(cx, cy, ax, ay)
    m = ((e0 >= 0) & (e1 >= 0) & (e2 >= 0)) | ((e0 <= 0) & (e1 <= 0) & (e2 <= 0))
    img[y0:y1, x0:x1][m] = color


def _goal(img, gx, gy):
    v = [(gx + dx, gy + dy) for dx, dy in GOAL_POLY]
    for k in range(1, len(v) - 1):   # GL_POLYGON as a triangle fan from vertex 0
        _triangle(img, (v[0], v[k], v[k + 1]), BLACK)


def draw(cfg, agent, goal, statics, dynamics) -> np.ndarray:
    """The reference viewer's frame for one env as an (H, W, 3) uint8 array, top row first."""
    img = np.full((cfg.screen_height, cfg.screen_width, 3), 255, np.uint8)
    _disk(img, agent[0], agent[1], cfg.radius_agent, BLACK)
    _goal(img, goal[0], goal[1])
    for p in statics:
        _disk(img, p[0], p[1], cfg.radius_obstacle, RED)
    for p in dynamics:
        _disk(img, p[0], p[1], cfg.radius_obstacle, GREEN)
    return img[::-1].copy()  # y up


def rgb_array(env, index: int = 0) -> np.ndarray:
    cfg = env.cfg
    return draw(cfg, env.agent[index].tolist(), env.goal[index].tolist(),
                env.static_obs[:cfg.num_static, index].tolist(), env.dyn_obs[:cfg.num_dynamic, index].tolist())


def render_env0(env, mode: str = "rgb_array"):
    img = rgb_array(env, 0)
    if mode == "rgb_array":
        return img
    if mode == "human":
        try:
            import pygame
        except ImportError as e:
            raise RuntimeError("render(mode='human') needs pygame; use mode='rgb_array'") from e
        if not pygame.display.get_init():
            pygame.display.init()
        surf = pygame.display.set_mode((img.shape[1], img.shape[0]))
        pygame.surfarray.blit_array(surf, img.swapaxes(0, 1))
        pygame.display.flip()
        pygame.event.pump()
        return None
    raise ValueError(f"unknown render mode {mode!r}")
