"""Deterministic synthetic inputs; there is no dataset on the GPU box.

ScanNet-crop clouds mimic the geometry of the reference's training crops
(attention_points/scannet_dataset/data_transformation.py:98-151): a 1.9 x 1.9 m footprint
(1.5 m crop + 0.2 m context margin each side) by 3 m height holding 12,000 unique surface
points — 40 % floor, 30 % two walls, 30 % faces of three boxes, +-5 mm jitter — from which
8192 points are drawn WITH replacement (data_transformation.py:145), so duplicate points
and therefore exact FPS / ball-query ties are present, as in the reference's training data.
Features are rgb/255 (train.py:95) and unit surface normals, 6 channels.

Random numbers: counter-based SplitMix64 with seed 0x5EED + cloud_id, float = (u >> 40) * 2^-24,
so any rank can generate any cloud of a global batch without communication.
"""
import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
SEED_BASE = 0x5EED


def splitmix64(seed, n, offset=0):
    """n outputs of SplitMix64 starting at state seed + offset*gamma (counter form)."""
    i = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def uniform(seed, n, offset=0):
    """U[0,1) with 24-bit resolution, float64 (exactly representable in float32)."""
    return (splitmix64(seed, n, offset) >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


def scannet_crop(cloud_id, n_points=8192, n_unique=12000, with_features=True):
    """One synthetic ScanNet crop: xyz (n_points,3) float32 and features (n_points,6) float32
    (rgb/255, normal), or None without features."""
    seed = SEED_BASE + int(cloud_id)
    u = uniform(seed, 16 * n_unique + n_points + 64)
    pos = [0]

    def take(k):
        a = u[pos[0]:pos[0] + k]
        pos[0] += k
        return a

    W, H = 1.9, 3.0
    n_floor = int(0.4 * n_unique)
    n_wall = int(0.15 * n_unique)
    n_box = n_unique - n_floor - 2 * n_wall
    pts, nrm = [], []
    # floor z = 0
    pts.append(np.stack([W * take(n_floor), W * take(n_floor), np.zeros(n_floor)], 1))
    nrm.append(np.tile([0.0, 0.0, 1.0], (n_floor, 1)))
    # wall x = 0 and wall y = 0
    pts.append(np.stack([np.zeros(n_wall), W * take(n_wall), H * take(n_wall)], 1))
    nrm.append(np.tile([1.0, 0.0, 0.0], (n_wall, 1)))
    pts.append(np.stack([W * take(n_wall), np.zeros(n_wall), H * take(n_wall)], 1))
    nrm.append(np.tile([0.0, 1.0, 0.0], (n_wall, 1)))
    # three boxes standing on the floor; points on their 5 visible faces
    box = take(3 * 5)
    per = [n_box // 3, n_box // 3, n_box - 2 * (n_box // 3)]
    for bi in range(3):
        cx, cy = 0.3 + 1.3 * box[5 * bi], 0.3 + 1.3 * box[5 * bi + 1]
        sx, sy, sz = 0.2 + 0.6 * box[5 * bi + 2], 0.2 + 0.6 * box[5 * bi + 3], 0.3 + 0.9 * box[5 * bi + 4]
        k = per[bi]
        face = np.minimum((take(k) * 5).astype(np.int64), 4)
        a, b = take(k), take(k)
        x = cx + (a - 0.5) * sx
        y = cy + (b - 0.5) * sy
        z = a * sz
        n = np.zeros((k, 3))
        p = np.zeros((k, 3))
        # 0:+x 1:-x 2:+y 3:-y 4:+z
        m = face == 0; p[m] = np.stack([np.full(m.sum(), cx + sx / 2), y[m], z[m]], 1); n[m] = [1, 0, 0]
        m = face == 1; p[m] = np.stack([np.full(m.sum(), cx - sx / 2), y[m], z[m]], 1); n[m] = [-1, 0, 0]
        m = face == 2; p[m] = np.stack([x[m], np.full(m.sum(), cy + sy / 2), b[m] * sz], 1); n[m] = [0, 1, 0]
        m = face == 3; p[m] = np.stack([x[m], np.full(m.sum(), cy - sy / 2), b[m] * sz], 1); n[m] = [0, -1, 0]
        m = face == 4; p[m] = np.stack([x[m], y[m], np.full(m.sum(), sz)], 1); n[m] = [0, 0, 1]
        pts.append(p)
        nrm.append(n)
    pts = np.concatenate(pts, 0)
    nrm = np.concatenate(nrm, 0)
    pts = pts + (take(3 * n_unique).reshape(n_unique, 3) - 0.5) * 0.01  # +-5 mm jitter
    rgb = np.floor(take(3 * n_unique).reshape(n_unique, 3) * 256.0) / 255.0
    pick = np.minimum((take(n_points) * n_unique).astype(np.int64), n_unique - 1)  # with replacement
    xyz = pts[pick].astype(np.float32)
    if not with_features:
        return xyz, None
    feats = np.concatenate([rgb, nrm], 1)[pick].astype(np.float32)
    return xyz, feats


def uniform_cloud(cloud_id, n_points):
    """Uniform control cloud U[0,1)^3 (the reference tests' randomf(), query_ball_point.cpp:9)."""
    return uniform(SEED_BASE + int(cloud_id), 3 * n_points).reshape(n_points, 3).astype(np.float32)


def batch(cloud_ids, n_points=8192, kind="scannet", with_features=False):
    """Stack clouds: xyz (B,N,3) float32 and features (B,N,6) or None."""
    xs, fs = [], []
    for cid in cloud_ids:
        if kind == "scannet":
            x, f = scannet_crop(cid, n_points, with_features=with_features)
        elif kind == "uniform":
            x, f = uniform_cloud(cid, n_points), None
        else:
            raise ValueError(kind)
        xs.append(x)
        fs.append(f)
    xyz = np.stack(xs, 0)
    feats = np.stack(fs, 0) if with_features and kind == "scannet" else None
    return xyz, feats


def features_uniform(seed, shape):
    """U[-1,1) float32 tensor standing in for an MLP output."""
    n = int(np.prod(shape))
    return (uniform(seed, n) * 2.0 - 1.0).astype(np.float32).reshape(shape)


def scannet_scene(scene_id, n_points=60000, size=(6.0, 4.5, 2.6)):
    """A synthetic ScanNet-like room (the input of the crop sampler / scene chunker,
    scannet_dataset/data_transformation.py:70, complete_scene_loader.py:4): floor, four walls
    and a few boxes, points (n,3) float32 with the room's corner at a random offset, labels
    (n,) int32 in [0, 20] (0 = unannotated, ~15 %), colours (n,3) int32 in [0, 255], unit
    normals (n,3) float32. Deterministic in scene_id."""
    import numpy as np
    g = np.random.default_rng(0xC0FFEE + scene_id)
    sx, sy, sz = size
    kind = g.choice(3, n_points, p=[0.35, 0.35, 0.30])
    pts = np.empty((n_points, 3), np.float64)
    nrm = np.zeros((n_points, 3), np.float64)
    lab = np.empty(n_points, np.int64)
    f = kind == 0  # floor
    pts[f] = np.stack([g.uniform(0, sx, f.sum()), g.uniform(0, sy, f.sum()), np.zeros(f.sum())], 1)
    nrm[f, 2] = 1
    lab[f] = 2
    w = kind == 1  # walls
    side = g.integers(0, 4, w.sum())
    t = g.uniform(0, 1, w.sum())
    z = g.uniform(0, sz, w.sum())
    wx = np.where(side == 0, t * sx, np.where(side == 1, t * sx, np.where(side == 2, 0.0, sx)))
    wy = np.where(side == 0, 0.0, np.where(side == 1, sy, t * sy))
    pts[w] = np.stack([wx, wy, z], 1)
    nrm[w] = np.stack([(side == 2) * 1.0 - (side == 3) * 1.0, (side == 0) * 1.0 - (side == 1) * 1.0,
                       np.zeros(w.sum())], 1)
    lab[w] = 1
    b = kind == 2  # boxes (furniture)
    nb = 6
    cx, cy = g.uniform(0.5, sx - 0.5, nb), g.uniform(0.5, sy - 0.5, nb)
    hx, hy, hz = g.uniform(0.2, 0.6, nb), g.uniform(0.2, 0.6, nb), g.uniform(0.4, 1.2, nb)
    bi = g.integers(0, nb, b.sum())
    u, v = g.uniform(-1, 1, b.sum()), g.uniform(-1, 1, b.sum())
    face = g.integers(0, 3, b.sum())
    px = np.where(face == 0, cx[bi] + np.sign(u) * hx[bi], cx[bi] + u * hx[bi])
    py = np.where(face == 1, cy[bi] + np.sign(v) * hy[bi], cy[bi] + v * hy[bi])
    pz = np.where(face == 2, 2 * hz[bi], g.uniform(0, 1, b.sum()) * 2 * hz[bi])
    pts[b] = np.stack([px, py, pz], 1)
    nrm[b, 2] = 1
    lab[b] = 3 + bi % 18
    pts += g.normal(0, 0.005, pts.shape)
    pts += g.uniform(-3, 3, 3) * np.array([1, 1, 0.1])
    lab[g.uniform(0, 1, n_points) < 0.15] = 0
    col = g.integers(0, 256, (n_points, 3)).astype(np.int32)
    return (pts.astype(np.float32), lab.astype(np.int32), col,
            (nrm / np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-9)).astype(np.float32))
