"""Window-attention output of one libvclip.so build on a test case, saved for comparison:
  python tools/win_diag.py <lib> <out.npy> [case] [qmul]"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from vclip_amd import _lib  # noqa: E402
_lib.load(sys.argv[1])
import test_swin3d_gpu as T  # noqa: E402
cases = [(2, (4, 6, 6), 32, (2, 3, 3), (0, 0, 0)), (2, (4, 6, 6), 64, (2, 3, 3), (1, 1, 1))]
B, grid, C, window, shift = cases[int(sys.argv[3]) if len(sys.argv) > 3 else 1]
qmul = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
if qmul != 1.0:
    B, grid, C, window, shift = 1, (4, 6, 6), 64, (2, 3, 3), (1, 1, 1)
got, want = T._window_case(B, grid, C, window, shift, seed=11 if qmul != 1.0 else C + sum(shift), qmul=qmul)
np.save(sys.argv[2], got.numpy())
np.save(sys.argv[2].replace(".npy", "_want.npy"), want.numpy())
print(sys.argv[1], "qmul", qmul, "max err", (got - want).abs().max().item(), "mean err", (got - want).abs().mean().item())
