"""dlrm_hip — MI355X-native (gfx950) DLRM training hot path.

Drop-in mirror of the reference's DLRM_Net surface (YuxinxinChen/dlrm-yx,
dlrm_s_pytorch.py:226-989) backed by hand-written CDNA4 HIP kernels behind the C-ABI in
include/dlrm_hip.h (libdlrm_hip.so, built in-tree).  No CPU fallback: every compute op
raises if the HIP library is missing.
"""
from ._lib import DLRMHipError, DLRMHipUnavailable, load as load_library  # noqa: F401

__version__ = "0.1.0"
