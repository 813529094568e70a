"""a reference ViViT checkpoint (transformers-4.48.2 key names inside the trainer's
dict, vivit_transformer/vivit_classifier/trainers/trainer.py:291-305) loads into the build.

The 4.48 names are written out here from the 4.48 module tree (encoder.layer.N.attention.attention.
{query,key,value}, attention.output.dense, intermediate.dense, output.dense).  The installed
transformers-5 library is the judge of the renaming: its own `from_pretrained` loads a checkpoint
saved with those names (its conversion_mapping ViTModel rules, which VivitModel uses), and
vclip_amd.checkpoint.convert_state_dict must produce exactly the state dict it produces."""
import json
import os
import re

import pytest
import torch

transformers = pytest.importorskip("transformers")

CFG = dict(image_size=32, num_frames=4, tubelet_size=[2, 16, 16], num_channels=3, hidden_size=128,
           num_hidden_layers=2, num_attention_heads=2, intermediate_size=128, hidden_act="gelu_fast",
           layer_norm_eps=1e-6, qkv_bias=True)

_TO_448 = [  # transformers-5 name -> 4.48.2 name (test data, from the 4.48 module structure)
    (r"\.layers\.(\d+)\.attention\.q_proj\.", r".encoder.layer.\1.attention.attention.query."),
    (r"\.layers\.(\d+)\.attention\.k_proj\.", r".encoder.layer.\1.attention.attention.key."),
    (r"\.layers\.(\d+)\.attention\.v_proj\.", r".encoder.layer.\1.attention.attention.value."),
    (r"\.layers\.(\d+)\.attention\.o_proj\.", r".encoder.layer.\1.attention.output.dense."),
    (r"\.layers\.(\d+)\.mlp\.fc1\.", r".encoder.layer.\1.intermediate.dense."),
    (r"\.layers\.(\d+)\.mlp\.fc2\.", r".encoder.layer.\1.output.dense."),
    (r"\.layers\.(\d+)\.", r".encoder.layer.\1."),
]


def _to_448(k):
    for a, b in _TO_448:
        if re.search(a, k):
            return re.sub(a, b, k)
    return k


@pytest.fixture(scope="module")
def hf_pair(tmp_path_factory):
    from transformers import VivitConfig, VivitForVideoClassification
    torch.manual_seed(0)
    cfg = VivitConfig(**CFG, id2label={0: "non-referral", 1: "referral"})
    m5 = VivitForVideoClassification(cfg).eval()
    sd5 = {k: v.detach().clone() for k, v in m5.state_dict().items()}
    old = {_to_448(k): v for k, v in sd5.items()}
    assert any("encoder.layer.1.attention.attention.query.weight" in k for k in old)
    d = tmp_path_factory.mktemp("vivit448")
    from safetensors.torch import save_file
    save_file(old, str(d / "model.safetensors"))
    cfg.save_pretrained(str(d))
    m_loaded = VivitForVideoClassification.from_pretrained(str(d)).eval()
    return sd5, old, {k: v.detach() for k, v in m_loaded.state_dict().items()}


def test_hf_itself_loads_the_448_names(hf_pair):
    sd5, old, loaded = hf_pair
    assert set(loaded) == set(sd5)
    for k in sd5:
        assert torch.equal(loaded[k], sd5[k]), k


def test_convert_state_dict_matches_hf_conversion(hf_pair):
    from vclip_amd.checkpoint import convert_state_dict
    sd5, old, loaded = hf_pair
    got = convert_state_dict(old)
    assert set(got) == set(loaded)
    for k in loaded:
        assert torch.equal(got[k], loaded[k]), k
    # DataParallel prefix (videoswintransformer/inference.py:73-87 strips it)
    got_dp = convert_state_dict({"module." + k: v for k, v in old.items()})
    assert set(got_dp) == set(loaded)


def test_reference_training_checkpoint_dict_loads(hf_pair, tmp_path):
    """The dict schema trainer.py:291-305 writes, read back weights-only, renamed, and loaded into
    the build's model (whose hf_state_dict uses the transformers-5 names)."""
    from vclip_amd.checkpoint import load_reference_checkpoint
    from vclip_amd.vivit import VivitConfig, VivitForVideoClassification
    sd5, old, loaded = hf_pair
    ck = {"epoch": 3, "model_state_dict": old, "optimizer_state_dict": {}, "val_loss": 0.5, "val_acc": 0.75,
          "history": {"train_loss": [1.0]}, "config": dict(CFG, id2label={0: "non-referral", 1: "referral"}),
          "id2label": {0: "non-referral", 1: "referral"}, "label2id": {"non-referral": 0, "referral": 1},
          "num_frames": 4, "train_sampling": "uniform", "val_sampling": "uniform", "test_sampling": "uniform"}
    path = tmp_path / "best_model_uniform.pth"
    torch.save(ck, path)
    ck2, sd = load_reference_checkpoint(str(path))
    assert ck2["epoch"] == 3 and ck2["id2label"] == {0: "non-referral", 1: "referral"}
    model = VivitForVideoClassification(VivitConfig(**CFG, id2label={0: "non-referral", 1: "referral"}))
    model.load_state_dict(sd)
    mine = model.hf_state_dict()
    for k in loaded:
        assert torch.equal(mine[k].detach().cpu(), loaded[k]), k
    json.dumps(ck2["config"])
    assert os.path.exists(path)
