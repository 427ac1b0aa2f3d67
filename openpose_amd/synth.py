"""Synthetic BODY_25 inputs: people overlays (heatmaps + PAFs), net input frames, weights.

There are no trained weights or datasets in this environment, so every workload is
synthetic and deterministic in a seed:

* ``people(n, h, w, seed)``      -- n skeletons in BODY_25 layout inside an h x w map
* ``render_field(...)``          -- net-output-like field [78, h, w]: 25 Gaussian heatmaps, the
  background channel, and 26 unit-vector PAF strips, laid out exactly as the reference's
  net_output blob (heatmaps, background, PAFs indexed by POSE_MAP_INDEX;
  /root/reference/src/openpose/pose/poseParameters.cpp:253-256, bodyPartConnectorBase.cpp:299-302)
* ``he_weights(layers, seed)``   -- per-layer seeded He-normal conv weights, zero bias, PReLU 0.25
"""
import numpy as np

from .pose_tables import BODY25_PAIRS, BODY25_MAP_IDX

# approximate BODY_25 skeleton in a unit-height box centred on the mid hip (x right, y down)
_TEMPLATE = np.array([
    (0.00, -0.42), (0.00, -0.32), (-0.12, -0.31), (-0.16, -0.15), (-0.18, 0.00),
    (0.12, -0.31), (0.16, -0.15), (0.18, 0.00), (0.00, 0.02), (-0.07, 0.02),
    (-0.08, 0.24), (-0.08, 0.45), (0.07, 0.02), (0.08, 0.24), (0.08, 0.45),
    (-0.03, -0.45), (0.03, -0.45), (-0.06, -0.43), (0.06, -0.43), (0.11, 0.50),
    (0.13, 0.49), (0.07, 0.47), (-0.11, 0.50), (-0.13, 0.49), (-0.07, 0.47)], np.float64)


def people(n, h, w, seed, min_height=0.35, max_height=0.9):
    """n random skeletons [n, 25, 2] (x, y) in pixel units of an h x w map."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 25, 2), np.float64)
    for p in range(n):
        ph = h * rng.uniform(min_height, max_height) / max(1.0, np.sqrt(n) / 2)
        cx = rng.uniform(0.1 * w, 0.9 * w)
        cy = rng.uniform(0.3 * h, 0.7 * h)
        pts = _TEMPLATE * ph + (cx, cy)
        pts += rng.normal(0, ph * 0.01, pts.shape)
        out[p] = pts
    return out


BODY25_TABLE = dict(id=0, name="BODY_25", parts=25, bkg=True, pairs=list(BODY25_PAIRS),
                    map_idx=list(BODY25_MAP_IDX))


def tree_template(table):
    """Unit-height skeleton [parts, 2] for any pose model: the parts laid out breadth-first along
    the model's pair graph from part pairs[0] (fixed directions, shrinking steps).  Only the
    topology matters for the synthetic workloads (the PAF of every pair runs from A to B)."""
    P = table["parts"]
    pairs = table["pairs"]
    adj = [[] for _ in range(P)]
    for q in range(len(pairs) // 2):
        a, b = pairs[2 * q], pairs[2 * q + 1]
        adj[a].append(b)
        adj[b].append(a)
    pos = np.full((P, 2), np.nan)
    depth = np.zeros(P, np.int64)
    order = [pairs[0]]
    pos[pairs[0]] = (0.0, -0.3)
    golden = np.pi * (3 - np.sqrt(5))
    k = 0
    while order:
        nxt = []
        for u in order:
            for v in adj[u]:
                if np.isnan(pos[v, 0]):
                    k += 1
                    depth[v] = depth[u] + 1
                    step = 0.16 / np.sqrt(depth[v])
                    th = golden * k
                    pos[v] = pos[u] + step * np.array([np.cos(th), 0.6 * np.abs(np.sin(th)) + 0.2])
                    nxt.append(v)
        order = nxt
    missing = np.isnan(pos[:, 0])   # parts outside every pair: spread below the root
    pos[missing] = np.stack([np.linspace(-0.2, 0.2, missing.sum()), np.full(missing.sum(), 0.45)], 1) \
        if missing.any() else pos[missing]
    return pos


def people_model(table, n, h, w, seed, min_height=0.35, max_height=0.9):
    """n random skeletons [n, parts, 2] of any pose model (BODY_25: people())."""
    if table["parts"] == 25 and list(table["pairs"]) == list(BODY25_PAIRS):
        return people(n, h, w, seed, min_height, max_height)
    tpl = tree_template(table)
    rng = np.random.default_rng(seed)
    out = np.zeros((n, table["parts"], 2), np.float64)
    for p in range(n):
        ph = h * rng.uniform(min_height, max_height) / max(1.0, np.sqrt(n) / 2)
        cx = rng.uniform(0.1 * w, 0.9 * w)
        cy = rng.uniform(0.3 * h, 0.7 * h)
        out[p] = tpl * ph + (cx, cy) + rng.normal(0, ph * 0.01, tpl.shape)
    return out


def render_field(skeletons, h, w, sigma, paf_width, background=True, table=None):
    """Render the net_output layout [parts + bkg + PAFs, h, w] float32 of a pose model (default
    BODY_25: [78, h, w]) from skeletons [n, parts, 2]."""
    t = table or BODY25_TABLE
    P, npairs = t["parts"], len(t["pairs"]) // 2
    base = P + (1 if t["bkg"] else 0)
    field = np.zeros((base + len(t["map_idx"]), h, w), np.float32)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    rad = int(np.ceil(4 * sigma))
    for sk in skeletons:
        for k in range(P):
            x, y = sk[k]
            x0, x1 = max(0, int(x) - rad), min(w, int(x) + rad + 2)
            y0, y1 = max(0, int(y) - rad), min(h, int(y) + rad + 2)
            if x0 >= x1 or y0 >= y1:
                continue
            d2 = (xx[y0:y1, x0:x1] - x) ** 2 + (yy[y0:y1, x0:x1] - y) ** 2
            g = np.exp(-d2 / (2 * sigma * sigma)).astype(np.float32)
            np.maximum(field[k, y0:y1, x0:x1], g, out=field[k, y0:y1, x0:x1])
    if background and t["bkg"]:
        field[P] = 1.0 - field[:P].max(axis=0)
    count = np.zeros((npairs, h, w), np.float32)
    for sk in skeletons:
        for q in range(npairs):
            a, b = sk[t["pairs"][2 * q]], sk[t["pairs"][2 * q + 1]]
            v = b - a
            length = float(np.hypot(*v))
            if length < 1e-6:
                continue
            u = v / length
            x0 = max(0, int(min(a[0], b[0]) - paf_width - 1))
            x1 = min(w, int(max(a[0], b[0]) + paf_width + 2))
            y0 = max(0, int(min(a[1], b[1]) - paf_width - 1))
            y1 = min(h, int(max(a[1], b[1]) + paf_width + 2))
            if x0 >= x1 or y0 >= y1:
                continue
            px = xx[y0:y1, x0:x1] - a[0]
            py = yy[y0:y1, x0:x1] - a[1]
            along = px * u[0] + py * u[1]
            across = np.abs(px * u[1] - py * u[0])
            m = (along >= 0) & (along <= length) & (across <= paf_width)
            cx = base + t["map_idx"][2 * q]
            cy = base + t["map_idx"][2 * q + 1]
            field[cx, y0:y1, x0:x1][m] += u[0]
            field[cy, y0:y1, x0:x1][m] += u[1]
            count[q, y0:y1, x0:x1][m] += 1
    for q in range(npairs):
        c = np.maximum(count[q], 1)
        field[base + t["map_idx"][2 * q]] /= c
        field[base + t["map_idx"][2 * q + 1]] /= c
    return field


def overlay(n_people, h, w, seed, table=None):
    """Net-output-resolution overlay: sigma 1 px Gaussians, 1 px PAF strips."""
    t = table or BODY25_TABLE
    return render_field(people_model(t, n_people, h, w, seed), h, w, sigma=1.0, paf_width=1.0,
                        table=t)


def fnv1a(name):
    h = 0xcbf29ce484222325
    for ch in name.encode():
        h ^= ch
        h = (h * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def he_weights(layers, seed=0, out_scale=1.0):
    """Seeded He-normal weights per conv layer: {name: (w [co,ci,k,k], bias [co], slope [co]|None)}.

    ``layers`` is the list of layer dicts of ``openpose_amd.graph`` (or oracle.body25).  The seed of
    a layer is FNV-1a(layer name) ^ seed.  ``out_scale`` multiplies the weights of the last conv of
    every stage (the Mconv7 layers) -- used to keep the synthetic net output small so a people
    overlay dominates post-processing.
    """
    params = {}
    slopes = {l["bottom"][0]: True for l in layers if l.get("type") == "PReLU"}
    for l in layers:
        if l.get("type", "Convolution") != "Convolution":
            continue
        if l.get("act") == 2:
            slopes[l["name"]] = True
        l = dict(l, top=l.get("top", [l["name"]]))
        rng = np.random.default_rng(fnv1a(l["name"]) ^ seed)
        co, ci, k = l["num_output"], l["cin"], l["kernel_size"]
        std = np.sqrt(2.0 / (ci * k * k))
        wt = rng.normal(0.0, std, (co, ci, k, k)).astype(np.float32)
        if l["name"].startswith("Mconv7"):
            wt *= np.float32(out_scale)
        b = np.zeros(co, np.float32)
        s = np.full(co, 0.25, np.float32) if l["top"][0] in slopes else None
        params[l["name"]] = (wt, b, s)
    return params
