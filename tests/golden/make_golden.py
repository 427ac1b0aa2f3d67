"""Generate the committed golden fixtures under tests/golden/ (run in the build container).

    PYTHONPATH=. python tests/golden/make_golden.py

connector_*.npz  -- expected keypoints/scores computed by the REFERENCE's own connector code
                    (bodyPartConnectorBase.cpp compiled from /root/reference into oracle/_ref);
                    inputs are regenerated from the stored seeds (openpose_amd.synth is
                    deterministic) and checked against the stored SHA-256 of the field and peaks.
nms_*.npz, resize_*.npz, cnn_*.npz
                 -- outputs of the oracle's CPU restatements (parity unpinned: the reference code
                    behind them needs OpenCV / Caffe, absent from the image); stored so the GPU box
                    (no /root/reference) checks the same numbers and regressions are caught.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
from oracle import body25  # noqa: E402
from openpose_amd import synth  # noqa: E402
from tests.fields import noise_field, people_field  # noqa: E402

CONNECTOR_CASES = [  # (name, kind, n_people, seed, h, w, maximize_positives)
    ("p1", "people", 1, 101, 368, 656, False),
    ("p5", "people", 5, 102, 368, 656, False),
    ("p20", "people", 20, 103, 368, 656, False),
    ("p0", "people", 0, 104, 368, 656, False),
    ("p5_small", "people", 5, 105, 184, 328, False),
    ("p5_maxpos", "people", 5, 106, 368, 656, True),
    ("noise", "noise", 0, 107, 120, 160, False),
]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def connector_field(kind, n, seed, h, w):
    if kind == "people":
        return people_field(n, h, w, seed)
    f = noise_field(78, h, w, seed, levels=6, density=0.7)
    f[26:] = f[26:] * 2 - 1
    return f


def make_connector():
    assert oracle.ref_lib() is not None, "needs /root/reference (oracle/_ref)"
    for name, kind, n, seed, h, w, maxpos in CONNECTOR_CASES:
        f = connector_field(kind, n, seed, h, w)
        scale = 1.959128
        off = np.float32(0.5 / scale)
        pk = oracle.nms(f, 0.05, 128, (off, off))
        kw = dict(scale=scale, maximize_positives=maxpos)
        kp, ks = oracle.connect(f, pk, use_reference=True, **kw)
        np.savez_compressed(os.path.join(HERE, "connector_%s.npz" % name), kind=kind, n_people=n,
                            seed=seed, h=h, w=w, maximize_positives=maxpos, scale=scale,
                            field_sha=sha(f), peaks=pk, keypoints=kp, scores=ks)


# connectBodyPartsGpu host assembly (GPU semantics), any model: (name, model, kind, n, seed, h, w,
# maximize_positives).  kind "people": synthetic field -> oracle NMS -> oracle pair scores;
# "random": random peaks and random pair scores (many merges and fragments).  The "_noface"
# BODY_135 cases blank the face parts; the "_face" cases keep them and are checked to reach the
# reference's face-fragment merge (removePeopleBelowThresholdsAndFillFaces with the restated
# getKeypointsRoi, oracle/ref_driver.cpp; round 5).
GPU_CONNECTOR_CASES = [
    ("b25_p5", 0, "people", 5, 111, 368, 656, False),
    ("b25_p20", 0, "people", 20, 112, 368, 656, False),
    ("b25_random", 0, "random", 0, 113, 368, 656, False),
    ("b135_p3", 14, "people_noface", 3, 114, 184, 328, False),
    ("b135_p8", 14, "people_noface", 8, 115, 368, 656, False),
    ("b135_p8_maxpos", 14, "people_noface", 8, 116, 368, 656, True),
    ("b135_random", 14, "random_noface", 0, 117, 184, 328, False),
    ("b25b_p6", 13, "people", 6, 118, 184, 328, False),
    ("b135_p3_face", 14, "people", 3, 131, 184, 328, False),
    ("b135_p8_face", 14, "people", 8, 132, 368, 656, False),
    ("b135_random_face", 14, "random", 0, 133, 184, 328, False),
    ("b135_random_face_maxpos", 14, "random", 0, 134, 184, 328, True),
]


def gpu_connector_inputs(table, kind, n, seed, h, w):
    """(peaks [parts,128,3], dense pair scores [npairs,127,127]) of one GPU-connector case.
    kind "people_noface": BODY_135 people whose face heat maps are blanked (no face peaks)."""
    if kind.startswith("people"):
        t = table
        sk = synth.people_model(t, n, h, w, seed)
        sc = h / 368.0
        f = synth.render_field(sk, h, w, sigma=max(1.0, 7.0 * sc), paf_width=max(1.0, 6.0 * sc),
                               table=t)
        if kind == "people_noface":
            f[65:t["parts"]] = 0
        scale = 1.959128
        off = np.float32(0.5 / scale)
        pk = oracle.nms(f, 0.05, 128, (off, off), channels=t["parts"])
        return pk, oracle.pair_scores_table(f, pk, t)
    rng = np.random.default_rng(seed)
    P, npairs = table["parts"], len(table["pairs"]) // 2
    pk = np.zeros((P, 128, 3), np.float32)
    for k in range(P):
        c = 0 if (kind == "random_noface" and k >= 65) else int(rng.integers(0, 5))
        pk[k, 0, 0] = c
        pk[k, 1:c + 1, 0] = rng.uniform(0, w, c)
        pk[k, 1:c + 1, 1] = rng.uniform(0, h, c)
        pk[k, 1:c + 1, 2] = rng.uniform(0.05, 1.0, c)
    ps = np.zeros((npairs, 127, 127), np.float32)
    for q in range(npairs):
        na, nb = int(pk[table["pairs"][2 * q], 0, 0]), int(pk[table["pairs"][2 * q + 1], 0, 0])
        v = rng.uniform(-0.5, 1.0, (na, nb)).astype(np.float32)
        ps[q, :na, :nb] = np.where(v > 0.2, v, 0)
    return pk, ps


def sparse_scores(ps):
    q, i, j = np.nonzero(ps)
    return np.stack([q, i, j], 1).astype(np.int16), ps[q, i, j].astype(np.float32)


def dense_scores(idx, val, npairs):
    ps = np.zeros((npairs, 127, 127), np.float32)
    ps[idx[:, 0], idx[:, 1], idx[:, 2]] = val
    return ps


def make_connector_gpu():
    assert oracle.ref_lib() is not None, "needs /root/reference (oracle/_ref)"
    tables = oracle.pose_tables()
    for name, model, kind, n, seed, h, w, maxpos in GPU_CONNECTOR_CASES:
        t = tables[model]
        pk, ps = gpu_connector_inputs(t, kind, n, seed, h, w)
        res = oracle.connect_gpu_semantics(ps, pk, t, use_reference=True, scale=1.959128,
                                           maximize_positives=maxpos)
        if name.endswith(("_face", "_face_maxpos")):
            assert oracle.face_merge_reached(ps, pk, t, maximize_positives=maxpos), \
                name + ": does not reach the face-fragment merge; pick another seed"
        idx, val = sparse_scores(ps)
        np.savez_compressed(os.path.join(HERE, "gpuconn_%s.npz" % name), model=model, kind=kind,
                            n_people=n, seed=seed, h=h, w=w, maximize_positives=maxpos,
                            scale=1.959128, peaks=pk, score_idx=idx, score_val=val,
                            npairs=len(t["pairs"]) // 2, keypoints=res[0], scores=res[1])
        print(name, "peaks", int(pk[:, 0, 0].sum()), "scores", len(val), "people", len(res[1]))


def make_nms():
    cases = {"people": people_field(5, 92, 164, 201),
             "noise": noise_field(78, 40, 56, 202, levels=5, density=0.8),
             "plateau": noise_field(78, 33, 35, 203, levels=3, density=1.0)}
    for name, f in cases.items():
        pk = oracle.nms(f, 0.05, 128, (0.25, 0.5))
        np.savez_compressed(os.path.join(HERE, "nms_%s.npz" % name), field=f, peaks=pk)


def make_resize():
    rng = np.random.default_rng(301)
    src = rng.normal(0, 0.5, (2, 10, 20)).astype(np.float32)
    out = oracle.resize_merge([src], 80, 160)
    srcs = [rng.normal(0, 0.5, (2, h, w)).astype(np.float32) for h, w in [(10, 20), (7, 15), (5, 10)]]
    merged = oracle.resize_merge(srcs, 80, 160)
    # a target width that is not a multiple of OpenCV's 4-float vertical SIMD vector (2 tail
    # columns summed left to right), and the OpenCV 3.x order for comparison (resize.c)
    rsrc = rng.normal(0, 0.5, (2, 9, 21)).astype(np.float32)
    rout = oracle.resize_merge([rsrc], 72, 166)
    with oracle.resize_order("3.x"):
        out3 = oracle.resize_merge([src], 80, 160)
    np.savez_compressed(os.path.join(HERE, "resize.npz"), src=src, out=out,
                        ms_src0=srcs[0], ms_src1=srcs[1], ms_src2=srcs[2], ms_out=merged,
                        ragged_src=rsrc, ragged_out=rout, out_opencv3=out3)


def make_cnn():
    graph = body25.layers()
    params = synth.he_weights(graph, seed=401)
    x = np.random.default_rng(402).uniform(-0.5, 0.5, (1, 3, 64, 96)).astype(np.float32)
    out = body25.forward(x, params, graph=graph)
    np.savez_compressed(os.path.join(HERE, "cnn_body25_64x96.npz"), weight_seed=401,
                        input=x, net_output=out)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()["make_" + name]()
        sys.exit(0)
    make_connector()
    make_connector_gpu()
    make_nms()
    make_resize()
    make_cnn()
    print("fixtures written to", HERE)
