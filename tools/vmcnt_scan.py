"""List, per kernel of a HIP source, the loops whose body waits on vmcnt before its first MFMA while
also issuing global loads (a prefetch the compiler's wait may drain every iteration: round 5 found
this in the attention backward and the conv_c path).  Static: reads the device assembly.
  python tools/vmcnt_scan.py ai-laryngeal-video-based-classifier_amd/csrc/attention.hip [...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ai-laryngeal-video-based-classifier_amd")


def asm(src):
    out = os.path.join("/tmp", os.path.basename(src) + ".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(PKG, "csrc"), "--cuda-device-only", "-S", src, "-o", out],
                   check=True, capture_output=True)
    return open(out).read()


def scan(text):
    for m in re.finditer(r"^(_Z\w+):", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        lines = [ln.split(";")[0].strip() for ln in text[m.end():end].split("\n")]
        labels = {}
        for i, ln in enumerate(lines):
            lm = re.match(r"^(\.LBB\w+):", ln)
            if lm:
                labels[lm.group(1)] = i
        for i, ln in enumerate(lines):
            bm = re.match(r"^s_cbranch_\w+\s+(\.LBB\w+)", ln) or re.match(r"^s_branch\s+(\.LBB\w+)", ln)
            if not bm or labels.get(bm.group(1), i + 1) > i:
                continue
            body = lines[labels[bm.group(1)]:i + 1]
            loads = sum(1 for b in body if b.startswith(("global_load", "buffer_load")) and "lds" not in b)
            first_mfma = next((k for k, b in enumerate(body) if b.startswith("v_mfma")), None)
            waits = [b for b in body[:first_mfma] if b.startswith("s_waitcnt") and "vmcnt" in b] if first_mfma else []
            if loads and waits:
                print(f"{name[:80]}: loop of {len(body)} lines, {loads} register loads, waits before the first "
                      f"MFMA: {', '.join(w.replace('s_waitcnt ', '') for w in waits[:6])}")


for src in sys.argv[1:]:
    print("==", src)
    scan(asm(src))
