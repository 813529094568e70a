"""Extract the argparse flags of the reference CLIs (read as text with `ast`, nothing imported)
into tests/golden/cli_flags.json: {"<folder>/<script>": {flag: {type, default, required, choices,
action}}}.  tests/test_cli_cpu.py checks vclip_amd.apps' parsers against it."""
import ast
import json
import os
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "cli_flags.json")
SCRIPTS = [f"{d}/{s}.py" for d in ("vivit_transformer", "timesformer", "videoswintransformer", "resnet50-3d-video")
           for s in ("main", "inference")]


def lit(node):
    try:
        return ast.literal_eval(node)
    except Exception:
        return ast.unparse(node)


def flags(path):
    out = {}
    for n in ast.walk(ast.parse(open(path).read())):
        if isinstance(n, ast.Call) and getattr(n.func, "attr", None) == "add_argument":
            name = lit(n.args[0])
            kw = {k.arg: lit(k.value) for k in n.keywords if k.arg in ("type", "default", "required", "choices", "action")}
            out[name] = kw
    return out


if __name__ == "__main__":
    res = {s: flags(os.path.join(REF, s)) for s in SCRIPTS}
    json.dump(res, open(OUT, "w"), indent=1, sort_keys=True)
    print(OUT, sum(len(v) for v in res.values()), "flags", file=sys.stderr)
