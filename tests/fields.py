"""Deterministic test fields for the post-processing stages."""
import numpy as np

from openpose_amd import synth


def people_field(n, h, w, seed, sigma=None, paf_width=None):
    """[78, h, w] BODY_25 net-output-layout field with n synthetic people."""
    scale = h / 368.0
    sigma = sigma if sigma is not None else max(1.0, 7.0 * scale)
    paf_width = paf_width if paf_width is not None else max(1.0, 6.0 * scale)
    return synth.render_field(synth.people(n, h, w, seed), h, w, sigma=sigma, paf_width=paf_width)


def noise_field(c, h, w, seed, levels=8, density=0.5):
    """Quantised noise: many local maxima, plateaus (ties) and border peaks."""
    rng = np.random.default_rng(seed)
    f = rng.integers(0, levels, (c, h, w)).astype(np.float32) / np.float32(levels - 1)
    f *= (rng.random((c, h, w)) < density).astype(np.float32)
    return f


def smooth_noise_field(c, h, w, seed):
    """Smooth random field (values in ~[-1, 1]) -- a net-output-like input for resize tests."""
    rng = np.random.default_rng(seed)
    return rng.normal(0, 0.5, (c, h, w)).astype(np.float32)
