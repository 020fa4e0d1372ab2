"""Shared parity tolerances.

fp32 forward: abs 1e-6.  Gradients: rel 1e-4 / abs 1e-7 (summation order differs).
Post-Adam parameters: abs 1e-6, EXCEPT the 'sign-flip zone': at Adam's first steps the update
is ~ lr * g/(|g|+eps), so an element whose effective gradient g + wd*p is below ZONE is driven by
fp32 summation noise (e.g. user_product_attention.k_proj.bias, whose true gradient is exactly 0
because softmax is shift-invariant over keys).  Those elements may differ by <= 2*lr per step.
"""
import numpy as np

ZONE = 1e-6


def assert_params_close(name, actual, ref, g_eff0, lr, steps, atol=1e-6):
    actual = np.asarray(actual, np.float32)
    ref = np.asarray(ref, np.float32)
    d = np.abs(actual - ref)
    zone = np.abs(g_eff0) < ZONE
    out_bad = (d > atol) & ~zone
    assert not out_bad.any(), (f"{name}: {out_bad.sum()} elements outside the sign-flip zone "
                               f"differ by up to {d[out_bad].max():.3e}")
    in_bad = d[zone]
    if in_bad.size:
        assert in_bad.max() <= 2 * lr * steps + atol, f"{name}: zone diff {in_bad.max():.3e}"


def assert_moment_close(name, actual, ref, g_eff0, rtol=1e-3, atol=1e-7):
    """Adam moments after a few steps.  exp_avg is (1-b1) * sum_k b1^k g_k (weights summing to
    < 0.3 over 3 steps), so it inherits the gradient tolerance scaled down: abs 1e-7 (the gradient
    abs tolerance is 1e-6), rel 1e-3 for elements accumulated from noisy near-zero gradients."""
    actual = np.asarray(actual)
    ref = np.asarray(ref)
    zone = np.abs(g_eff0) < ZONE
    d = np.abs(actual - ref)
    bad = (d > atol + rtol * np.abs(ref)) & ~zone
    assert not bad.any(), f"{name}: {bad.sum()} moment elements differ (max {d[bad].max():.3e})"
