"""Drop-in for the reference's `resnet50-3d-video/inference.py` (same flags): runs on libvclip / MI355X.

    python cli/resnet50-3d-video/inference.py <the reference's arguments>
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vclip_amd.apps import run_inference  # noqa: E402

if __name__ == "__main__":
    run_inference("resnet3d")
