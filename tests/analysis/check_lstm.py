"""[tools experiment, outside the product suite: python -m pytest tests/analysis/check_lstm.py after
python tools/lstm_gpu/build.py]  ResNet50-LSTM on the GPU vs oracle/lstm_ref.py (torch's own nn.LSTM for the recurrence; the
ResNet-50 part restates torchvision, which is absent: UNPINNED there).  Logit tolerance 1e-2."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools", "lstm_gpu"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lstm_model  # noqa: E402

from oracle.lstm_ref import lstm_forward
from vclip_amd.weights import make_resnet50_lstm_weights, make_synthetic_video

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vclip_amd import _lib
    _lib.load()


def test_lstm_recurrence_vs_torch():
    g = torch.Generator().manual_seed(0)
    B, T, Hs, Din = 3, 8, 256, 64
    lstm = torch.nn.LSTM(Din, Hs, batch_first=True)
    x = torch.randn(B, T, Din, generator=g)
    with torch.no_grad():
        want, _ = lstm(x)
        pre = x.reshape(B * T, Din) @ lstm.weight_ih_l0.T + lstm.bias_ih_l0 + lstm.bias_hh_l0
    hseq = torch.zeros(B * T, Hs, dtype=torch.bfloat16, device=DEV)
    hlast = torch.zeros(B, Hs, device=DEV)
    lstm_model.lstm_recurrence(pre.to(DEV), B, T, Hs, lstm.weight_hh_l0.detach().contiguous().to(DEV), hseq, hlast)
    assert (hlast.cpu() - want[:, -1]).abs().max().item() < 1e-5
    assert (hseq.float().cpu().view(B, T, Hs) - want).abs().max().item() < 8e-3  # bf16 copy


@pytest.mark.parametrize("B,T", [(1, 8), (2, 4)])
def test_resnet50_lstm_logits(B, T):
    from lstm_model import VideoResNet50LSTM
    w = make_resnet50_lstm_weights(seed=0)
    video = make_synthetic_video(B, T, 224, seed=7)
    with torch.no_grad():
        want = lstm_forward({k: torch.from_numpy(v) for k, v in w.items()}, torch.from_numpy(video)).numpy()
    m = VideoResNet50LSTM()
    m.load_state_dict(w)
    got = m.to(DEV)(torch.from_numpy(video).to(DEV)).cpu().numpy()
    assert np.abs(got - want).max() < 1e-2, (got, want)
