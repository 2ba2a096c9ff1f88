"""EnvConfig: the BallEnv knobs, with the reference's names and defaults.

Sources of each field (reference paths):
* module constants            gym_ballenv/envs/ballenv_env.py:11-18
* BallEnv.__init__ constants  gym_ballenv/envs/ballenv_env.py:47-65
* customize_environment(args) gym_ballenv/envs/ballenv_env.py:87-109, with the
  argparse defaults of examples/ball_cnn_ac3.py:37-59 and its checks :61-68
* move_list (9 actions)       examples/ball_cnn_ac3.py:530
* TimeLimit(1000)             gym_ballenv/__init__.py:4-11
"""
from __future__ import annotations

from dataclasses import dataclass, field, fields, replace
from typing import List, Tuple

from . import _abi

MOVE_LIST: List[Tuple[int, int]] = [(1, 1), (1, -1), (1, 0), (0, 1), (0, -1), (0, 0), (-1, 1), (-1, 0), (-1, -1)]
DEFAULT_GOALS: List[Tuple[int, int]] = [(12, 122), (123, 93), (87, 150), (430, 440), (230, 11)]


@dataclass
class EnvConfig:
    # field + spawn strips (ballenv_env.py:11-18)
    screen_width: int = 500
    screen_height: int = 500
    strip_obs_x: int = 0
    strip_obs_y: int = 20
    strip_goal_x: int = 500
    strip_goal_y: int = 20
    strip_agent_x: int = 500
    strip_agent_y: int = 10
    # BallEnv.__init__ (ballenv_env.py:47-65)
    radius_obstacle: int = 20        # radius_rand_person
    radius_agent: int = 5            # radius_ctrl_person
    speed_x: int = 1                 # speedx_ctrl_person (also prep_state4's cell step)
    speed_y: int = 1                 # speedy_ctrl_person
    threshold_goal: float = 10.0
    time_penalty: float = 0.0
    min_spawn_dist: float = 50.0     # reset re-sample distance (ballenv_env.py:122)
    # customize_environment(args) (ballenv_env.py:87-109; defaults ball_cnn_ac3.py:40-51)
    num_static: int = 13             # args.static_obstacles
    num_dynamic: int = 5             # args.dynamic_obstacles
    obstacle_speed: List[int] = field(default_factory=lambda: [1, 1, 1, 1, 1])
    goals: List[Tuple[int, int]] = field(default_factory=lambda: list(DEFAULT_GOALS))
    goal_change_step: int = 50       # args.time_step_for_change
    obs_certainty: int = 60          # args.rd_th_obs
    static_penalty: float = 1.0      # args.static_penalty[1] (threshold_2_penalty)
    dynamic_penalty: float = 8000.0  # args.dynamic_penalty[1]
    # action table (ball_cnn_ac3.py:530) and episode handling
    actions: List[Tuple[int, int]] = field(default_factory=lambda: list(MOVE_LIST))
    time_limit: int = 1000           # gym TimeLimit; 0 = none
    autoreset: bool = True

    @classmethod
    def from_args(cls, args, base: "EnvConfig | None" = None) -> "EnvConfig":
        """customize_environment(args) (ballenv_env.py:87-109), same field names.

        Applies the assert_arguments checks of ball_cnn_ac3.py:61-68 and, like the
        reference, uses index [1] of the threshold/penalty pairs.
        """
        c = replace(base) if base is not None else cls()
        nd = int(args.dynamic_obstacles)
        speeds = [int(s) for s in args.obstacle_speed]
        goals = []
        for tup in args.obs_goal_position:
            x, y = tup.strip().split(",")[:2]
            goals.append((int(x), int(y)))
        if len(speeds) != nd:
            raise AssertionError("The length of the list of obstacle_speed does not match the no. of dynamic obstacles")
        if len(goals) != nd:
            raise AssertionError("The length of the list of obstacle_goal_position does not match the no. of dynamic obstacles")
        for name in ("static_penalty", "dynamic_penalty"):
            if len(getattr(args, name)) != 2:
                raise AssertionError(f"The length of the list of {name} is not equal to 2")
        c.num_static = int(args.static_obstacles)
        c.num_dynamic = nd
        c.obstacle_speed = speeds
        c.goals = goals
        c.goal_change_step = int(args.time_step_for_change)
        c.obs_certainty = int(args.rd_th_obs)
        c.static_penalty = float(args.static_penalty[1])
        c.dynamic_penalty = float(args.dynamic_penalty[1])
        return c

    def to_abi(self, num_envs: int, window: int, env_offset: int = 0, seed: int = 0xBA11) -> _abi.BeConfig:
        b = _abi.BeConfig()
        b.num_envs, b.window, b.env_offset, b.seed = int(num_envs), int(window), int(env_offset), int(seed) & (2**64 - 1)
        for f in ("screen_width", "screen_height", "strip_obs_x", "strip_obs_y", "strip_goal_x", "strip_goal_y",
                  "strip_agent_x", "strip_agent_y", "radius_obstacle", "radius_agent", "speed_x", "speed_y",
                  "num_static", "num_dynamic", "goal_change_step", "obs_certainty", "time_limit"):
            setattr(b, f, int(getattr(self, f)))
        for f in ("threshold_goal", "time_penalty", "min_spawn_dist", "static_penalty", "dynamic_penalty"):
            setattr(b, f, float(getattr(self, f)))
        if len(self.goals) > _abi.MAX_GOALS or len(self.obstacle_speed) > _abi.MAX_DYNAMIC \
                or len(self.actions) > _abi.MAX_ACTIONS:
            raise ValueError("too many goals / obstacle speeds / actions for the C ABI")
        if len(self.obstacle_speed) < self.num_dynamic:
            raise ValueError("need one obstacle_speed per dynamic obstacle")
        b.num_goals = len(self.goals)
        for g, (x, y) in enumerate(self.goals):
            b.goals[g][0], b.goals[g][1] = int(x), int(y)
        for k, s in enumerate(self.obstacle_speed):
            b.obstacle_speed[k] = int(s)
        b.num_actions = len(self.actions)
        for a, (dx, dy) in enumerate(self.actions):
            b.actions[a][0], b.actions[a][1] = int(dx), int(dy)
        b.autoreset = 1 if self.autoreset else 0
        return b

    def validate(self, num_envs: int, window: int) -> None:
        msg = _abi.config_check(self.to_abi(num_envs, window))
        if msg:
            raise ValueError(msg)

    def as_dict(self) -> dict:
        return {f.name: getattr(self, f.name) for f in fields(self)}


def step_bytes(cfg: EnvConfig, window: int) -> int:
    """Algorithmic HBM bytes per env-step of the step kernel."""
    return _abi.step_bytes(cfg.to_abi(1, window))



def survey_step_bytes(cfg: EnvConfig, window: int) -> int:
    """SURVEY.md §8(d)'s algorithmic bytes per env-step (the roofline's per-unit figure).

    It prices the step-API traffic of the reference's natural SoA layout:
    int32 coordinates, a stored per-obstacle counter and a u8 obs,
    ``82 + 8*Ns + 20*Nd + (4 + W^2)`` = 390 B at Ns=13, Nd=5, W=10.
    ``step_bytes`` is what this engine's packed layout actually moves (275 B there).
    """
    return 82 + 8 * cfg.num_static + 20 * cfg.num_dynamic + 4 + window * window
