"""Configuration records, field-compatible with the reference's
`tauv_vision.centernet.model.config` (config.py:6-196) so existing configs and
`to_dict`/`from_dict` round trips carry over unchanged."""
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Tuple


@dataclass
class ModelConfig:
    """config.py:6-35. Output grid = input // 2**downsamples."""
    backbone_heights: List[int]
    backbone_channels: List[int]
    in_h: int
    in_w: int
    downsamples: int
    angle_bin_overlap: float

    @property
    def downsample_ratio(self) -> int:
        return 1 << self.downsamples

    @property
    def out_h(self) -> int:
        return self.in_h // self.downsample_ratio

    @property
    def out_w(self) -> int:
        return self.in_w // self.downsample_ratio

    def to_dict(self):
        return asdict(self)

    @classmethod
    def from_dict(cls, data):
        return cls(**data)


@dataclass
class TrainConfig:
    """config.py:38-69 (carried for config-file compatibility; training is out of scope)."""
    lr: float
    batch_size: int
    n_batches: int
    n_epochs: int
    heatmap_focal_loss_a: float
    heatmap_focal_loss_b: float
    heatmap_sigma_factor: float
    keypoint_heatmap_sigma: float
    keypoint_affinity_sigma: float
    loss_lambda_keypoint_heatmap: float
    loss_lambda_keypoint_affinity: float
    loss_lambda_size: float
    loss_lambda_offset: float
    loss_lambda_angle: float
    loss_lambda_depth: float
    n_workers: int
    weight_save_interval: int

    def to_dict(self):
        return asdict(self)

    @classmethod
    def from_dict(cls, data):
        return cls(**data)


@dataclass
class AngleConfig:
    """config.py:72-82."""
    train: bool
    modulo: Optional[float]

    def to_dict(self):
        return asdict(self)

    @classmethod
    def from_dict(cls, data):
        return cls(**data)


@dataclass
class ObjectConfig:
    """config.py:85-120: one detectable object class."""
    id: str
    yaw: AngleConfig
    pitch: AngleConfig
    roll: AngleConfig
    train_depth: bool
    train_keypoints: bool
    keypoints: Optional[List[Tuple[float, float, float]]]

    def to_dict(self):
        d = {"id": self.id, "train_depth": self.train_depth, "train_keypoints": self.train_keypoints}
        for axis in ("yaw", "pitch", "roll"):
            d[axis] = getattr(self, axis).to_dict()
        d["keypoints"] = None if self.keypoints is None else [list(k) for k in self.keypoints]
        return d

    @classmethod
    def from_dict(cls, data):
        kps = data["keypoints"]
        return cls(id=data["id"], yaw=AngleConfig.from_dict(data["yaw"]), pitch=AngleConfig.from_dict(data["pitch"]),
                   roll=AngleConfig.from_dict(data["roll"]), train_depth=data["train_depth"],
                   train_keypoints=data["train_keypoints"],
                   keypoints=None if kps is None else [tuple(k) for k in kps])


class ObjectConfigSet:
    """config.py:124-196: the label set; keypoints are numbered object by object, slot by
    slot, skipping objects without keypoints."""

    def __init__(self, configs: List[ObjectConfig]):
        self.configs: List[ObjectConfig] = configs
        self._kp_to_flat: Dict[Tuple[int, int], int] = {}
        self._flat_to_kp: Dict[int, Tuple[int, int]] = {}
        for obj, cfg in enumerate(configs):
            for slot in range(len(cfg.keypoints or [])):
                flat = len(self._flat_to_kp)
                self._kp_to_flat[(obj, slot)] = flat
                self._flat_to_kp[flat] = (obj, slot)

    def to_dict(self):
        return {"object_configs": [c.to_dict() for c in self.configs]}

    @classmethod
    def from_dict(cls, data):
        return cls(configs=[ObjectConfig.from_dict(c) for c in data["object_configs"]])

    @property
    def train_yaw(self) -> bool:
        return any(c.yaw.train for c in self.configs)

    @property
    def train_pitch(self) -> bool:
        return any(c.pitch.train for c in self.configs)

    @property
    def train_roll(self) -> bool:
        return any(c.roll.train for c in self.configs)

    @property
    def train_depth(self) -> bool:
        return any(c.train_depth for c in self.configs)

    @property
    def train_keypoints(self) -> bool:
        return any(c.train_keypoints for c in self.configs)

    @property
    def n_labels(self) -> int:
        return len(self.configs)

    @property
    def n_keypoints(self) -> int:
        return len(self._flat_to_kp)

    @property
    def label_id_to_index(self) -> Dict[str, int]:
        return {c.id: i for i, c in enumerate(self.configs)}

    def encode_keypoint_index(self, object_index: int, object_keypoint_index: int) -> int:
        return self._kp_to_flat[(object_index, object_keypoint_index)]

    def decode_keypoint_index(self, keypoint_index) -> Tuple[int, int]:
        return self._flat_to_kp[keypoint_index]

    def get_by_label(self, label: str) -> ObjectConfig:
        return self.configs[self.label_id_to_index[label]]
