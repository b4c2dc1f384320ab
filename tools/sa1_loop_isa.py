#!/usr/bin/env python3
"""Static instruction mix of the SA1 sampler's iteration loop in the built libpn2hip.so
(the loop place_sa1_loop.py places), written as JSON for bench.py's per-CU VALU bound:

    python tools/sa1_loop_isa.py [--lib pointcloud-segmentation-attention_amd/libpn2hip.so]
                                 [--out profiles/r1/sa1_loop_isa.json]

One iteration issues every instruction of the loop body once per wave (the body has no inner
loop; the t == 0 stores are EXEC-masked, still issued). With one wave per SIMD, a wave64 VALU
instruction occupies its SIMD for 4 cycles, so 4 x (VALU instructions) is the iteration's
VALU-issue floor; bench.py divides it by the measured cycles per iteration."""
import argparse
import json
import os
import re
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import place_sa1_loop  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "pointcloud-segmentation-attention_amd",
                                                  "libpn2hip.so"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r1", "sa1_loop_isa.json"))
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        start, body = place_sa1_loop.loop_body(args.lib, tmp)
    mix = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "branch": 0, "other": 0}
    for l in body:
        op = re.match(r"\s+([a-z_0-9]+)", l).group(1)
        if op.startswith("v_"):
            mix["valu"] += 1
        elif op.startswith(("s_cbranch", "s_branch")):
            mix["branch"] += 1
        elif op.startswith("s_"):
            mix["salu"] += 1
        elif op.startswith("ds_"):
            mix["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            mix["vmem"] += 1
        else:
            mix["other"] += 1
    out = {"kernel": "fps_v9_kernel<256, 32, 4, true, false, true, false, PAD> (SA1 sampler)",
           "loop_start_mod_64": start % 64, "instructions": len(body), "mix": mix,
           "valu_issue_floor_cycles": 4 * mix["valu"],
           "note": "static count of the iteration loop body; one wave per SIMD, 4 cycles per "
                   "wave64 VALU instruction"}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
