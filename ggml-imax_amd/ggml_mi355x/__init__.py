"""MI355X-native ggml runtime (Python side: ctypes mirror of the C API + helpers).

The product is the pair of shared libraries built from ../csrc (see ../Makefile):
lib/libggml_core.so (ggml API) and lib/libggml_mi355x.so (gfx950 backend).
"""
from . import ggml, synth  # noqa: F401

__all__ = ["ggml", "synth"]
