"""ops/wt_cache.py optimizer-driven W^T cache (CPU: the validity rules)."""
import torch

from distributed_model_parallel_amd.ops import wt_cache


def test_global_cache_tracks_optimizer_steps_and_versions():
    wt_cache.set_enabled(True)
    w = torch.nn.Parameter(torch.randn(24, 16, 1, 1).bfloat16())
    s0 = wt_cache.stats()
    t0 = wt_cache.transposed(w)  # miss: registers the weight
    assert torch.equal(t0, w.detach().reshape(24, 16).t())
    assert wt_cache.stats()["miss"] == s0["miss"] + 1
    assert wt_cache.stats()["hit"] == s0["hit"]
    with torch.no_grad():
        w.data.mul_(2.0)  # an optimizer writing through raw pointers (no version bump)
    wt_cache.after_optimizer_step([w])  # ... then refreshing the cache
    t1 = wt_cache.transposed(w)
    assert wt_cache.stats()["hit"] == s0["hit"] + 1
    assert torch.equal(t1, w.detach().reshape(24, 16).t())
    with torch.no_grad():
        w.add_(1.0)  # an in-place change the cache did not see: version bump -> miss
    t2 = wt_cache.transposed(w)
    assert torch.equal(t2, w.detach().reshape(24, 16).t())
    assert wt_cache.stats()["hit"] == s0["hit"] + 1
    wt_cache.after_optimizer_step([w])
    assert torch.equal(wt_cache.transposed(w), w.detach().reshape(24, 16).t())
    assert wt_cache.stats()["hit"] == s0["hit"] + 2
    # a non-leaf (e.g. a DataParallel replica's broadcast weight) is never registered
    v = (w * 1.0)
    n0 = len(wt_cache._WANTED)
    wt_cache.transposed(v)
    assert len(wt_cache._WANTED) == n0
    # a weight no optimizer of ours owns (refreshed elsewhere) never gets an entry
    u = torch.nn.Parameter(torch.randn(16, 32).bfloat16())
    wt_cache.transposed(u)
    wt_cache.after_optimizer_step([w])
    h = wt_cache.stats()["hit"]
    wt_cache.transposed(u)
    assert wt_cache.stats()["hit"] == h


def test_global_cache_drops_freed_weights():
    import gc
    wt_cache.set_enabled(True)
    wt_cache.after_optimizer_step()  # prune whatever earlier tests left

    def register():
        w = torch.nn.Parameter(torch.randn(8, 40, 1, 1).bfloat16())
        wt_cache.transposed(w)
        wt_cache.after_optimizer_step([w])
        return len(wt_cache._GLOBAL)
    n = register()
    gc.collect()
    wt_cache.after_optimizer_step()
    assert len(wt_cache._GLOBAL) == n - 1


def test_flip_fallback_matches_torch_on_cpu():
    """The CPU form of the tap-wise flipped transpose (what the refresh falls
    back to without the extension) against the torch expression it replaces."""
    from distributed_model_parallel_amd.ops import wt_cache
    w = torch.randn(8, 6, 3, 3).contiguous(memory_format=torch.channels_last).half()
    src = wt_cache._flip_src(w)
    d = torch.empty(6, 9 * 8, dtype=w.dtype)
    wt_cache._native_transpose([src], [d], [-9])
    assert torch.equal(d, w.flip(2, 3).permute(1, 2, 3, 0).reshape(6, -1))
    d1 = torch.empty(6, 9 * 8, dtype=w.dtype)
    wt_cache._native_transpose([src], [d1], [9])
    assert torch.equal(d1, w.permute(1, 2, 3, 0).reshape(6, -1))
    assert wt_cache._flip_src(torch.randn(8, 6, 3, 3)) is None  # not channels-last: no storage view
