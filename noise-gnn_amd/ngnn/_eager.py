"""The eager two-layer SAGE stack's C++ autograd node (csrc/ngnn_eager.cpp).

A torch C++ extension, built in-tree by ``build()`` (``__graft_entry__.build()``
calls it) into ``ngnn/lib/eager/ngnn_eager.so`` and imported from there --
never rebuilt at run time (the GPU box runs the prebuilt file).  It takes the
libngnn entry points as addresses from ``ngnn._lib``, so the kernels it runs
are the ones the Python node runs.  ``load()`` returns None when the module
was not built (ngnn.fused then keeps its Python node: the same HIP launches,
more host time per step).
"""
from __future__ import annotations

import ctypes
import importlib.machinery
import importlib.util
import os

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(_HERE, "lib", "eager")
SO_PATH = os.path.join(BUILD_DIR, "ngnn_eager.so")
_SRC = os.path.join(os.path.dirname(_HERE), "csrc", "ngnn_eager.cpp")
_INC = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include")

_mod = None
_tried = False


def build() -> str:
    """Compile the extension into BUILD_DIR (torch.utils.cpp_extension,
    ninja; a C++ file: g++ against torch's headers).  Returns the .so path."""
    from torch.utils import cpp_extension
    os.makedirs(BUILD_DIR, exist_ok=True)
    cpp_extension.load(name="ngnn_eager", sources=[_SRC], extra_include_paths=[_INC],
                       extra_cflags=["-O2"], build_directory=BUILD_DIR, verbose=False)
    return SO_PATH


def load():
    """The built module (entry points bound), or None if it is absent."""
    global _mod, _tried
    if _tried:
        return _mod
    _tried = True
    if os.environ.get("NGNN_EAGER_EXT", "1") == "0" or not os.path.exists(SO_PATH):
        return None
    import torch  # noqa: F401  (the module links libtorch: load it first)
    loader = importlib.machinery.ExtensionFileLoader("ngnn_eager", SO_PATH)
    spec = importlib.util.spec_from_file_location("ngnn_eager", SO_PATH, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    lib = _lib.load()
    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    mod.init(addr(lib.ngnn_sage2_fwd), addr(lib.ngnn_sage2_bwd), addr(lib.ngnn_row_extent),
             addr(lib.ngnn_block_prefix_stats), addr(lib.ngnn_strerror))
    _mod = mod
    return _mod
