"""vclip_amd — MI355X-native video-clip classification hot path.

Frame sampling (host, bit-exact with the reference samplers) -> frame gather/normalise
-> tubelet embedding -> joint space-time attention encoder -> classifier head, with
every device op a hand-written HIP kernel for gfx950 behind the C-ABI in
include/vclip.h (libvclip.so).  See DESIGN.md.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(PKG_DIR)

__all__ = ["PKG_DIR", "REPO_ROOT"]
