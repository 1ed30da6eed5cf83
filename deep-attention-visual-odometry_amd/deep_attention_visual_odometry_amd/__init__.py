"""MI355X-native batched BFGS bundle-adjustment solver.

Drop-in for the hot path of jskinn/deep-attention-visual-odometry
(``autograd_solvers/`` BFGS + strong-Wolfe on the ``camera_model/`` +
``geometry/`` reprojection objective).  Compute runs in the gfx950 library
``_lib/libdava_ba.so`` (C ABI: include/dava_ba.h); there is no CPU path.
"""
from .autograd_solvers import BFGSSolver, line_search_wolfe_conditions
from .camera_model import RayAngleError, ReprojectionError, num_parameters, unpack_calibration_parameters
from .camera_model import PinholeCameraModelL1
from .data import CameraAndParametersDataset, CameraViewsAndPoints
from .geometry import LieRotation
from .scenes import make_scenes
from .solvers import BFGSCameraSolver, IOptimisableFunction, LineSearchStrongWolfeConditions

__all__ = [
    "BFGSSolver",
    "line_search_wolfe_conditions",
    "RayAngleError",
    "ReprojectionError",
    "num_parameters",
    "unpack_calibration_parameters",
    "make_scenes",
    "CameraAndParametersDataset",
    "CameraViewsAndPoints",
    # legacy IOptimisableFunction path (solvers/, camera_model/pinhole_camera_model_l1.py)
    "BFGSCameraSolver",
    "IOptimisableFunction",
    "LieRotation",
    "LineSearchStrongWolfeConditions",
    "PinholeCameraModelL1",
]
