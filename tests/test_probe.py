"""opk_probe_peaks: the measured ceilings bench.py reports beside its rooflines."""
import pytest


@pytest.mark.gpu
def test_probe_peaks_plausible():
    from openpose_amd.api import Context
    p = Context(0).probe_peaks()
    # dense fp16 MFMA: at most the 2.5 PFLOP/s nominal, and random operands never beat zeros by much
    assert 500 < p["mfma_fp16_random_tflops"] < 2600
    assert 500 < p["mfma_fp16_zero_tflops"] < 2600
    assert p["mfma_fp16_random_tflops"] < 1.05 * p["mfma_fp16_zero_tflops"]
    assert 1000 < p["hbm_read_gbs"] < 8500
    print(p)
