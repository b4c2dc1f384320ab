#!/usr/bin/env python3
"""Static view of the culled sampler's hot-pick loop (fps_cull.h, wave 0's certified picks):
compiles csrc/fps.hip to gfx950 assembly (or reads --asm), finds the loop that publishes a pick
(`s_lshl_b64 exec, 1, ...`) in the fps_hotcull_kernel instantiation matching --kernel, and
prints its basic blocks with instruction counts by kind. The common path of one pick is every
block except the tie path (equal maxima, a second wave reduction).

    python tools/hot_loop_isa.py [--kernel 'ILi8192ELb0ELi3ELi4ELi1E'] [--asm fps.s] [--json out]

One wave alone issues one instruction per ~4 cycles (MI355X_MICROARCH.md, 'vector-instruction
ISSUE cost'; s_nop included), so 4 x (common-path instructions) is the issue floor of a pick."""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pointcloud-segmentation-attention_amd", "csrc")


def compile_asm(out, defines=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-ffp-contract=off", "--cuda-device-only", "-S", "fps.hip", "-o", out]
    cmd += [f"-D{d}" for d in defines]
    subprocess.run(cmd, cwd=CSRC, check=True, stderr=subprocess.DEVNULL)


def kind(op):
    if op == "s_nop":
        return "nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def hot_loops(asm_text, kernel):
    """Every pick loop of the instantiation (one per publishing asm block)."""
    m = re.search(r"^(_Z\S*fps_hotcull_kernel\S*" + re.escape(kernel) + r"\S*):", asm_text, re.M)
    if not m:
        raise SystemExit(f"no fps_hotcull_kernel instantiation matching {kernel!r}")
    body = asm_text[m.end():asm_text.index(".Lfunc_end", m.end())]
    n = body.count("s_lshl_b64 exec, 1,")
    return [hot_loop(asm_text, kernel, k) for k in range(n)]


def hot_loop(asm_text, kernel, which=0):
    m = re.search(r"^(_Z\S*fps_hotcull_kernel\S*" + re.escape(kernel) + r"\S*):", asm_text, re.M)
    if not m:
        raise SystemExit(f"no fps_hotcull_kernel instantiation matching {kernel!r}")
    body = asm_text[m.end():asm_text.index(".Lfunc_end", m.end())].split("\n")
    blocks, cur = [], None
    for line in body:
        lab = re.match(r"^(\.LBB\w+|; %bb\.\d+):", line)
        if lab:
            cur = {"label": lab.group(1), "ins": []}
            blocks.append(cur)
            continue
        ins = re.match(r"^\s+([a-z_][a-z_0-9]*)\b", line)
        if ins and cur is not None and not line.strip().startswith(";"):
            cur["ins"].append(line.strip())
    # the publishing block and the loop around it: from the loop header (the latest label
    # before it that a later branch jumps back to) to that back edge
    pubs = [i for i, b in enumerate(blocks) if any("s_lshl_b64 exec, 1," in x for x in b["ins"])]
    pub = pubs[which]
    for h in range(pub, -1, -1):
        lab = blocks[h]["label"]
        if not lab.startswith(".LBB"):
            continue
        back = [i for i in range(pub, len(blocks))
                if any(re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"$", x)
                       for x in blocks[i]["ins"])]
        if back:
            lo, hi = h, back[-1]
            break
    else:
        raise SystemExit("loop header not found")
    # the latch may sit before the header (rotated loops): include blocks that branch to the
    # header from before it
    pre = [i for i in range(0, lo) if any(re.search(r"s_c?branch\w*\s+" + re.escape(blocks[lo]["label"]) + r"$", x)
                                          for x in blocks[i]["ins"]) and i >= lo - 3]
    sel = list(range(min(pre + [lo]), hi + 1))
    out = []
    for i in sel:
        b = blocks[i]
        mix = {}
        for x in b["ins"]:
            k = kind(x.split()[0])
            mix[k] = mix.get(k, 0) + 1
        tie = any("v_max_u32_dpp" in x for x in b["ins"])
        out.append({"label": b["label"], "n": len(b["ins"]), "mix": mix, "tie_path": tie})
    common = sum(b["n"] for b in out if not b["tie_path"])
    return out, common


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="ILi16ELi9ELi8192ELb0ELi3ELi4ELi1E")
    ap.add_argument("--asm")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--json")
    ap.add_argument("--show", action="store_true", help="print the loop's instructions")
    args = ap.parse_args()
    if args.asm:
        text = open(args.asm).read()
    else:
        with tempfile.TemporaryDirectory() as tmp:
            path = os.path.join(tmp, "fps.s")
            compile_asm(path, args.D)
            text = open(path).read()
    loops = hot_loops(text, args.kernel)
    blocks, common = min(loops, key=lambda bc: bc[1])
    res = {"kernel": args.kernel, "loops": [c for _, c in loops], "blocks": blocks,
           "common_path_instructions": common, "issue_floor_cycles": 4 * common}
    if args.show:
        m = re.search(r"^(_Z\S*fps_hotcull_kernel\S*" + re.escape(args.kernel) + r"\S*):", text, re.M)
        body = text[m.end():text.index(".Lfunc_end", m.end())]
        first = body.index(blocks[0]["label"] + ":")
        last = body.index(blocks[-1]["label"] + ":") if blocks[-1]["label"].startswith(".LBB") \
            else body.index(blocks[-1]["label"])
        end = body.index("\n.LBB", last + 5)
        print(body[first:end])
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
