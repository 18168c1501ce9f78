"""MI355X-native host mirror of DROID-SLAM's update-operator path.

Mirrors the reference's Python interface for the hot path - CorrBlock /
AltCorrBlock (modules/corr.py), UpdateModule / ConvGRU / GraphAgg
(droid_net.py, modules/gru.py), DepthVideo (depth_video.py) and FactorGraph
(factor_graph.py) - on top of the `droid_backends` drop-in (HIP kernels via
the C ABI).  lietorch and torch_scatter are not needed.
"""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from .corr import AltCorrBlock, CorrBlock  # noqa: E402,F401
from .update import ConvGRU, GraphAgg, UpdateModule  # noqa: E402,F401
from .depth_video import DepthVideo  # noqa: E402,F401
from .factor_graph import FactorGraph  # noqa: E402,F401
from .extractor import BasicEncoder  # noqa: E402,F401
from .droid_net import DroidNet  # noqa: E402,F401
from .motion_filter import MotionFilter  # noqa: E402,F401
