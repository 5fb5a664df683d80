"""tauv_vision_amd — MI355X-native (gfx950) drop-in for TAUV-Vision's per-frame CenterNet
detection path: `Centernet(DLABackbone(...), object_config)(img) -> Prediction`, then
`decode` / `decode_keypoints`, with all compute in hand-written HIP kernels
(lib/libtauv_vision_amd.so, C ABI in include/tauv_vision_amd.h)."""
from .config import AngleConfig, ModelConfig, ObjectConfig, ObjectConfigSet, TrainConfig  # noqa: F401
from .centernet import (CenterpointDLA34, Centernet, Prediction, get_head_channels, initialize_weights,  # noqa: F401
                        preprocess)
from .dla import DLABackbone  # noqa: F401
from .decode import (Detection, KeypointDetection, angle_decode, angle_get_bins, decode,  # noqa: F401
                     decode_keypoints, decode_records, depth_decode, heatmap_detect, heatmap_nms)

__version__ = "0.1.0"
