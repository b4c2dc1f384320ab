#!/usr/bin/env python3
"""Diagnostic: the pipelined cfg2 step (3 sampler streams, layout b, native plan, direct
launches -- tests/test_gpu_a_fullsize.py's test_pipeline_full_size case) run for many
rotations over 3 buffer sets of distinct clouds, every set's outputs and index intermediates
compared bit for bit with the same clouds' eager step (stack.Step) after every rotation; the
sampled coordinates are poisoned before every other rotation (as the test does). Prints the
mismatches per rotation (which tensor, how many values)."""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rotations", type=int, default=30)
    ap.add_argument("--lanes", type=int, default=3)
    ap.add_argument("--layout", default="b")
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    S = pkg.stack
    dev = torch.device("cuda:0")
    B = 16
    sets = [S.make_inputs("cfg2", list(range(100 + i * B, 100 + (i + 1) * B)), dev) for i in range(3)]
    refs = []
    for inp in sets:
        st = S.Step(inp)
        outs = st()
        torch.cuda.synchronize()
        refs.append(([o.clone() for o in outs], {k: v.clone() for k, v in st.intermediates().items()}))
    pipe = S.Pipeline(sets[0], graphs=True, nsets=3, sampler_lanes=args.lanes, native_plan=True,
                      layout=args.layout, chain_own=False, set_inputs=sets, direct=True)
    bad = []
    for rot in range(args.rotations):
        if rot % 2 == 1:
            pipe.join()
            for s in pipe.sets:
                v = s.step.v
                for _, nx in (v.get("chain") or v.get("fps_out")):
                    nx.fill_(1e6)
            torch.cuda.synchronize()
        for _ in range(3):
            pipe.run()
        pipe.join()
        for si, (sinp, souts, sinter) in enumerate(pipe.outputs_by_set()):
            k = [i for i, x in enumerate(sets) if x is sinp]
            ro, ri = refs[k[0] if k else si]
            for i, (g, r) in enumerate(zip(souts, ro)):
                if not torch.equal(g.view(torch.int32) if g.dtype == torch.float32 else g,
                                   r.view(torch.int32) if r.dtype == torch.float32 else r):
                    bad.append({"rot": rot, "set": si, "out": i,
                                "n": int((g != r).sum().item())})
            for name, t in sinter.items():
                if not torch.equal(t, ri[name]):
                    bad.append({"rot": rot, "set": si, "inter": name,
                                "n": int((t != ri[name]).sum().item())})
    print(json.dumps({"rotations": args.rotations, "mismatches": len(bad), "first": bad[:30]}))


if __name__ == "__main__":
    main()
