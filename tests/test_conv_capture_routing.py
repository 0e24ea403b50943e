"""Round 4, profiles/README.md finding 48: inside a hipGraph capture the conv
routing leaves MIOpen out (its small-map weight gradient does not replay).
Since round 6 conv_wgrad_xl (the 4-wave TN tap gather) takes every Cin % 256
3x3 weight gradient eagerly too: it beats MIOpen's igemm_wrw at batch 2048
(the round-4 row cap is gone)."""
from distributed_model_parallel_amd.ops import conv_igemm


def test_xl_wgrad_gate(monkeypatch):
    monkeypatch.setattr(conv_igemm, "_XL_WGRAD", True)
    monkeypatch.setattr(conv_igemm, "_capturing", lambda: False)
    assert conv_igemm._xl_wgrad_ok(512, 3, 3, 12_544)       # layer 4 at batch 256
    assert conv_igemm._xl_wgrad_ok(512, 3, 3, 100_352)      # batch 2048: no longer MIOpen
    assert not conv_igemm._xl_wgrad_ok(128, 3, 3, 12_544)   # Cin % 256 != 0: not this kernel
    assert not conv_igemm._xl_wgrad_ok(512, 1, 1, 12_544)   # 1x1: the GEMM paths
    monkeypatch.setattr(conv_igemm, "_XL_WGRAD", False)
    assert not conv_igemm._xl_wgrad_ok(512, 3, 3, 12_544)   # DMP_DISABLE=xl_conv3


def test_generic_backward_env_default():
    # the generic native backward is opt-in eagerly (set_generic_backward); a
    # capture turns it on by itself
    assert conv_igemm.NATIVE_BWD in (False, True)
    assert callable(conv_igemm._capturing)
