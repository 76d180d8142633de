"""Defaults that the reference binds through gin (featurePnP/model.gin,
input_configs/*.gin: sparseFeaturePnP.*, optimize_feature_pnp.*).

gin is not part of this build; `configure()` sets the same bindings in-process.
"""
from . import losses

_MODEL = dict(n_iters=50, loss_fn=losses.squared_loss, lambda_=0.01, verbose=False, ratio_threshold=None,
              useGPU=True)  # featurePnP/model.gin:1-5
_ADAPTER = dict(image_shape=(1024, 1024), feature_pyramid=None)
# find_inliers.* (featurePnP/model.py:131; input_configs/robotcar_inlier_GN.gin:42 binds 0.8)
_FIND_INLIERS = dict(threshold=None, loss_fn=losses.squared_loss, mode="ratio_max")


def configure(**kwargs):
    """configure(n_iters=50, loss_fn=..., ratio_threshold=..., image_shape=..., feature_pyramid=...,
    find_inliers_threshold=..., find_inliers_loss_fn=..., find_inliers_mode=...)."""
    for k, v in kwargs.items():
        if k.startswith("find_inliers_"):
            k = k[len("find_inliers_"):]
            if k not in _FIND_INLIERS:
                raise KeyError(f"find_inliers has no parameter {k!r}")
            if isinstance(v, str) and k == "loss_fn":
                v = losses.by_name(v)
            _FIND_INLIERS[k] = v
        elif k in _ADAPTER:
            _ADAPTER[k] = v
        else:
            if isinstance(v, str) and k == "loss_fn":
                v = losses.by_name(v)
            _MODEL[k] = v


def model_kwargs():
    return dict(_MODEL)


def adapter_kwargs():
    return dict(_ADAPTER)


def find_inliers_kwargs():
    return dict(_FIND_INLIERS)
