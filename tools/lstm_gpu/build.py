"""Build tools/lstm_gpu/liblstm.so (the out-of-scope GPU ResNet50-LSTM recurrence experiment) for gfx950.
Not part of libvclip.so nor of __graft_entry__.build().   python tools/lstm_gpu/build.py"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def build():
    from vclip_amd.build import ARCH, CSRC, INCLUDE, _hipcc, _torch_libdir
    out = os.path.join(HERE, "liblstm.so")
    cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
           "-I", HERE, os.path.join(HERE, "lstm.hip"), "-o", out]
    tl = _torch_libdir()
    if tl:
        cmd += [f"-L{tl}", f"-Wl,-rpath,{tl}"]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    print(build())
