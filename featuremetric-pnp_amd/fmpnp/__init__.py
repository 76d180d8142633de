"""fmpnp -- MI355X-native feature-metric PnP refiner (drop-in for aunagar/FeatureMetric-PnP's
sparseFeaturePnP / feature_pnp / optimize_feature_pnp).  The compute path is libfmpnp.so
(HIP, gfx950); there is no CPU fallback."""
from . import _lib, config, losses, refine  # noqa: F401
from .losses import (barron, barron_loss, cauchy_loss, geman_mcclure_loss, huber_loss, scaled_loss,  # noqa: F401
                     squared_loss)
from .matrix_utils import matrix_quaternion  # noqa: F401
from .model import find_inliers, sparseFeaturePnP  # noqa: F401
from .optimize_feature_pnp import DirectPoseModel, feature_pnp, feature_pnp_multi, optimize_feature_pnp  # noqa: F401
from .refine import AsyncBatch, PackedFeatures, Problem, make_options, make_problem, pack_features  # noqa: F401
from . import cpu, pipeline, replay  # noqa: F401,E402
from .pipeline import RefinePipeline  # noqa: F401,E402

__version__ = "0.1.0"
