"""esmstereo_amd — MI355X-native (gfx950 HIP) ESMStereo hot path.

Drop-in for the reference ``models`` package on the hot path:

    from esmstereo_amd import __models__          # instead of `from models import __models__`
    model = __models__["ESMStereo"](192, gwc, norm_correlation, backbone, cv_scale)

Op-level drop-ins for ``models/submodule.py`` live in :mod:`esmstereo_amd.volumes`;
the ShuffleMixer blocks in :mod:`esmstereo_amd.mixer`; the hot-path modules in
:mod:`esmstereo_amd.blocks`.  Importing requires the in-tree ``libesmstereo_amd.so``
(build: ``python esmstereo_amd/build.py``); there is no CPU fallback.
"""
from ._lib import EsmError  # noqa: F401  (loads and checks the native library)
from .blocks import BasicConv, Conv2x, aggregation, up_refinement, upsample4, upsample8, upsample16  # noqa: F401
from .mixer import FMBlock, SMLayer, SplitPointMlp  # noqa: F401
from .model import ESMStereo, ESMStereo_confidence, ESMStereo_trt, FeatUp, HotPath  # noqa: F401
from .confidence import LAFNet_ESM, conf_upsample  # noqa: F401
from .volumes import (build_concat_volume, build_gwc_volume, build_norm_correlation_volume,  # noqa: F401
                      disparity_regression, regression_topk)

__models__ = {"ESMStereo": ESMStereo, "ESMStereo_trt": ESMStereo_trt, "ESMStereo_confidence": ESMStereo_confidence}

__version__ = "0.1.0"
