"""Drop-in for the reference's `videoswintransformer/main.py` (same flags): runs on libvclip / MI355X.

    python cli/videoswintransformer/main.py <the reference's arguments>
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vclip_amd.apps import run_main  # noqa: E402

if __name__ == "__main__":
    run_main("swin")
