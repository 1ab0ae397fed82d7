"""multimodaltraj_2_amd — MI355X-native (gfx950) implementation of the
g2k_lstm_mcr per-frame training path of serenetech90/multimodaltraj_2.

Host side: this package (PyTorch-ROCm for device memory / streams /
torch.distributed).  Compute: libg2k_hip.so, hand-written HIP kernels behind
the C ABI in include/g2k_hip.h.  See DESIGN.md.
"""
from ._lib import G2KError, G2KLibraryError, load as load_library  # noqa: F401

__all__ = ["G2KError", "G2KLibraryError", "load_library"]
