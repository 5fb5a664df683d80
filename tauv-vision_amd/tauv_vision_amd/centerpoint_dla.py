"""Drop-in `CenterpointDLA34` (reference src/tauv_vision/centernet/model/backbones/
centerpoint_dla.py:544-578), same module path tail as the reference."""
from .centernet import CenterpointDLA34  # noqa: F401
