"""ops/wt_cache.py: per-step W^T buffers shared by a pipeline step's
micro-batches (CPU: the cache logic; the GPU pipeline tests cover its use)."""
import torch

from distributed_model_parallel_amd.ops import wt_cache


def test_transposed_hits_after_refresh_and_tracks_updates():
    w = torch.nn.Parameter(torch.randn(24, 16, 1, 1))
    lin = torch.nn.Parameter(torch.randn(8, 12))
    c = wt_cache.WTCache([w, lin, torch.nn.Parameter(torch.randn(4, 4, 3, 3))])  # 3x3: not cached
    assert len(c) == 2
    assert torch.equal(wt_cache.transposed(w), w.detach().reshape(24, 16).t())  # inactive: a copy
    c.refresh()
    with c.active():
        h0 = wt_cache.stats()["hit"]
        t = wt_cache.transposed(w)
        assert wt_cache.stats()["hit"] == h0 + 1 and t.is_contiguous()
        assert torch.equal(t, w.detach().reshape(24, 16).t())
        assert torch.equal(wt_cache.transposed(lin), lin.detach().t())
        with torch.no_grad():
            w.mul_(2.0)  # an optimizer step between steps
        c.refresh()
        t2 = wt_cache.transposed(w)
        assert t2.data_ptr() == t.data_ptr()  # same storage: captured graphs stay valid
        assert torch.equal(t2, w.detach().reshape(24, 16).t())
        other = torch.randn(24, 16, 1, 1)
        m0 = wt_cache.stats()["miss"]
        assert torch.equal(wt_cache.transposed(other), other.reshape(24, 16).t())
        assert wt_cache.stats()["miss"] == m0 + 1
