"""Env configuration dataclasses: same field names and defaults as the reference's
(sokoban/config.py:4-21, frozen_lake/config.py:4-22, bandit/config.py:4-14,
countdown/config.py:5-11), so ``custom_envs.<tag>.env_config`` dicts load unchanged."""
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple


@dataclass
class SokobanEnvConfig:
    dim_room: Tuple[int, int] = (6, 6)
    max_steps: int = 100
    num_boxes: int = 3
    search_depth: int = 300
    grid_lookup: Optional[Dict[int, str]] = field(
        default_factory=lambda: {0: "#", 1: "_", 2: "O", 3: "√", 4: "X", 5: "P", 6: "S"})
    grid_vocab: Optional[Dict[str, str]] = field(default_factory=lambda: {
        "#": "wall", "_": "empty", "O": "target", "√": "box on target", "X": "box", "P": "player",
        "S": "player on target"})
    action_lookup: Optional[Dict[int, str]] = field(default_factory=lambda: {1: "Up", 2: "Down", 3: "Left", 4: "Right"})
    dim_x: Optional[int] = None
    dim_y: Optional[int] = None
    render_mode: str = "text"

    def __post_init__(self):
        if self.dim_x is not None and self.dim_y is not None:
            self.dim_room = (self.dim_x, self.dim_y)
        self.dim_room = tuple(int(x) for x in self.dim_room)


@dataclass
class FrozenLakeEnvConfig:
    size: int = 4
    p: float = 0.8
    is_slippery: bool = True
    map_seed: Optional[int] = None
    render_mode: str = "text"
    action_map: Dict[int, int] = field(default_factory=lambda: {1: 0, 2: 1, 3: 2, 4: 3})
    map_lookup: Dict[bytes, int] = field(default_factory=lambda: {b"P": 0, b"F": 1, b"H": 2, b"G": 3})
    grid_lookup: Dict[int, str] = field(default_factory=lambda: {0: "P", 1: "_", 2: "O", 3: "G", 4: "X", 5: "√"})
    grid_vocab: Dict[str, str] = field(default_factory=lambda: {
        "P": "player", "_": "empty", "O": "hole", "G": "goal", "X": "player in hole", "√": "player on goal"})
    action_lookup: Dict[int, str] = field(default_factory=lambda: {1: "Left", 2: "Down", 3: "Right", 4: "Up"})
    # gymnasium >= 1.1 slippery transition probabilities [(a-1)%4, a, (a+1)%4]
    success_rate: float = 1.0 / 3.0


@dataclass
class BanditEnvConfig:
    lo_arm_name: str = "phoenix"
    hi_arm_name: str = "dragon"
    action_space_start: int = 1
    lo_arm_score: float = 0.1
    hi_arm_loscore: float = 0.0
    hi_arm_hiscore: float = 1.0
    hi_arm_hiscore_prob: float = 0.25
    render_mode: str = "text"
    action_lookup: Dict[int, str] = None  # set per env at reset (bandit/env.py:37)


@dataclass
class CountdownEnvConfig:
    train_path: str = "data/countdown/train.parquet"
    max_instances: int = 20000
    render_mode: str = "text"
    score = 1
    format_score = 0.1
    # in-memory instances [{"nums": [...], "target": int}, ...] used instead of the parquet
    # (the reference's dataset is an HF download, absent offline)
    data: Optional[list] = None
