"""GPU parity of the whole-model step (stack.SemSegModel: pointnet2_sem_seg inference forward,
SA x4 + FP x4 + head, every MLP on the matrix cores) against a float64 CPU pipeline.

The pipeline uses the oracle for every INDEX (FPS, ball query, three_nn: bit-exact, pinned to
the reference in test_oracle_golden.py) and float64 numpy for every FLOAT (grouping, MLPs,
pooling, IDW interpolation). Tolerance (floating point, as in test_gpu_mlp.py):

    max |gpu - f64|  <=  max(4 * max |fp32 pipeline - f64|,  1e-6 * (1 + max |f64|))

where the fp32 pipeline is the same computation in numpy float32.
"""
import importlib

import numpy as np
import pytest

from conftest import PKG_NAME, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


def _mlp(x, layers, dt):
    y = np.asarray(x, dt)
    for L in layers:
        y = y @ L["weights"].astype(dt) + L["biases"].astype(dt)
        if "gamma" in L:
            s = L["gamma"].astype(np.float64) / np.sqrt(L["moving_variance"].astype(np.float64) + 1e-3)
            t = L["beta"].astype(np.float64) - L["moving_mean"].astype(np.float64) * s
            y = y * s.astype(dt) + t.astype(dt)
        if L["relu"]:
            y = np.maximum(y, 0)
    return y.astype(dt)


def pipeline(O, pkg, xyz, feats, store, dt):
    """pointnet2_sem_seg(_features) forward (pointnet2_sem_seg.py:29-60) in dtype dt, with the
    oracle's indices."""
    S = pkg.stack
    conv = lambda scope, cin, cout, bn=True, relu=True: {  # noqa: E731
        **{k: v.cpu().numpy() for k, v in store.conv(scope, cin, cout, bn=bn).items()}, "relu": relu}
    levels = [xyz]
    for (m, _, _, _) in S.SSG_SA:
        levels.append(O.gather_point(levels[-1], O.fps(levels[-1], m)))
    pts = [None if feats is None else feats.astype(dt)]
    c = 0 if feats is None else feats.shape[2]
    attention = store._packed and any(k[0] == "dense" for k in store._packed)
    for i, (m, r, ns, _) in enumerate(S.SSG_SA):
        idx, _ = O.ball_query(levels[i], levels[i + 1], r, ns)
        b = np.arange(xyz.shape[0])[:, None, None]
        gx = levels[i][b, idx].astype(dt) - levels[i + 1][:, :, None, :].astype(dt)
        g = gx if pts[i] is None else np.concatenate([gx, pts[i][b, idx]], axis=-1)
        layers = [conv(f"layer{i + 1}/conv{j}", c + 3 if j == 0 else S.SSG_SA_MLP[i][j - 1], w)
                  for j, w in enumerate(S.SSG_SA_MLP[i])]
        X = _mlp(g, layers, dt)
        c = S.SSG_SA_MLP[i][-1]
        if attention:  # attention_layer.py:29-45 + the batch norm of :261
            sc = f"layer{i + 1}"
            dq, dk, dv = [{**{k: v.cpu().numpy() for k, v in store.dense(d, c, c).items()},
                           "relu": False} for d in pkg.attention_layer._attention_scopes(sc)]
            Q = _mlp(X[:, :, 0], [dq], dt)
            K, V = _mlp(X, [dk], dt), _mlp(X, [dv], dt)
            Bm, Mm, nsm = X.shape[:3]
            H = c // 4
            Qh = Q.reshape(Bm, Mm, H, 1, 4)
            Kh = K.reshape(Bm, Mm, H, nsm, 4)  # the reference's reshape of (ns, C)
            Vh = V.reshape(Bm, Mm, H, nsm, 4)
            w = (Qh @ np.swapaxes(Kh, -1, -2)) / dt(2.0)
            w = np.exp(w - w.max(-1, keepdims=True))
            w = w / w.sum(-1, keepdims=True)
            out = (w @ Vh).reshape(Bm, Mm, c)
            bnp = {k: v.cpu().numpy() for k, v in store.bn(f"{sc}/{sc}", c).items()}
            s_ = bnp["gamma"].astype(np.float64) / np.sqrt(bnp["moving_variance"].astype(np.float64) + 1e-3)
            t_ = bnp["beta"].astype(np.float64) - bnp["moving_mean"].astype(np.float64) * s_
            pts.append((out * s_.astype(dt) + t_.astype(dt)).astype(dt))
        else:
            pts.append(X.max(axis=2))
    p2 = pts[4]
    for k, widths in enumerate(S.SSG_FP_MLP):
        lvl = 3 - k
        dist, nidx = O.three_nn(levels[lvl], levels[lvl + 1])
        r = 1.0 / np.maximum(dist.astype(dt), dt(1e-10))
        w = r / r.sum(axis=2, keepdims=True)
        b = np.arange(xyz.shape[0])[:, None, None]
        interp = (p2[b, nidx] * w[..., None]).sum(axis=2)
        x = interp if pts[lvl] is None else np.concatenate([interp, pts[lvl]], axis=-1)
        cin = x.shape[-1]
        layers = []
        for j, wd in enumerate(widths):
            layers.append(conv(f"fa_layer{k + 1}/conv_{j}", cin, wd))
            cin = wd
        if k == 3:
            layers.append(conv("fc1", cin, 128))
            layers.append(conv("fc2", 128, S.NUM_CLASSES, bn=False, relu=False))
        p2 = _mlp(x, layers, dt)
    return p2, pts[1:]


@pytest.mark.parametrize("config", ["cfg2", "cfg3"])
def test_model_step_vs_f64(config):
    import torch

    from oracle import oracle as O
    O.set_threads(16)
    pkg = importlib.import_module(PKG_NAME)
    dev = torch.device("cuda:0")
    inp = pkg.stack.make_inputs(config, [0, 1], dev, model=True)
    outs = pkg.stack.Step(inp)()
    torch.cuda.synchronize()
    logits = outs[0].cpu().numpy()
    assert logits.shape == (2, 8192, pkg.stack.NUM_CLASSES)
    xyz = inp["xyz"].cpu().numpy()
    feats = None if inp["feats"] is None else inp["feats"].cpu().numpy()
    store = inp["model"].store
    ref64, lv64 = pipeline(O, pkg, xyz, feats, store, np.float64)
    ref32, lv32 = pipeline(O, pkg, xyz, feats, store, np.float32)
    for got, r64, r32, what in [(logits, ref64, ref32, "logits")] + [
            (o.cpu().numpy(), a, b, f"l{i + 1}_points") for i, (o, a, b) in
            enumerate(zip(outs[1:], lv64, lv32))]:
        err = np.abs(got - r64).max()
        err32 = np.abs(r32 - r64).max()
        tol = max(4 * err32, 1e-6 * (1 + np.abs(r64).max()))
        assert np.isfinite(got).all()
        assert err <= tol, f"{config} {what}: err {err:.3g} > tol {tol:.3g} (fp32 {err32:.3g})"


def test_model_graph_replay_matches_eager():
    import torch
    pkg = importlib.import_module(PKG_NAME)
    dev = torch.device("cuda:0")
    inp = pkg.stack.make_inputs("cfg2", [3, 4], dev, model=True)
    eager = [o.clone() for o in pkg.stack.Step(inp)()]
    pipe = pkg.stack.Pipeline(inp, nsets=2)
    for _ in range(3):
        pipe.run()
    outs = pipe.join()
    for a, b in zip(eager, outs):
        assert torch.equal(a, b)
