"""k_paths' replay fast reject (csrc/avr_kernels.hip, the DDA walk's candidate test): inside the
DDA walk a free-flight candidate t = tMin + SampleExponential(u, sm0) (sampling.h:222-225,
media.h:770-777) is rejected WITHOUT evaluating the canonical log when

    A = sm0 * dt < 40  and  (1 - u) <= FastExp(-A) * (1 - 1e-3 - 5e-7 A),     dt = segMax - tMin

(FastExp being the factor T_maj needs anyway). The claim is exactness: every fast reject is a
reject of the canonical decision `!(tMin + SampleExponential(u, sm0) < segMax)`, so replay never
depends on the shortcut. Checked here on the host against the oracle's canonical-libm
SampleExponential and pbrt's FastExp (both pinned by the reference goldens), over random and
adversarial inputs concentrated at the decision boundary: large t (tMin up to 1e6), tiny and
huge dt, A up to and past 40, u within 1e-3 relative of the boundary."""
import numpy as np

from oracle import binding

f32 = np.float32


def _fast_reject(u, sm0, tMin, segMax):
    """The device expression in float32 (-ffp-contract=off, the k_paths build's flags)."""
    dt = f32(segMax - tMin)
    if np.isinf(dt):
        dt = f32(np.finfo(np.float32).max)
    A = f32(sm0 * dt)
    fac = f32(binding.lib().oracle_fastexp(float(-A)))
    bound = f32(fac * f32(f32(f32(1) - f32(1e-3)) - f32(f32(5e-7) * A)))
    return bool(A < f32(40) and f32(f32(1) - u) <= bound)


def _exact_reject(u, sm0, tMin, segMax):
    t = f32(tMin + f32(binding.lib().oracle_sample_exponential(float(u), float(sm0))))
    return not (t < segMax)


def test_every_fast_reject_is_an_exact_reject():
    binding.set_libm("canonical")
    rng = np.random.default_rng(5)
    n_fast = n_checked = 0
    try:
        for _ in range(60000):
            sm0 = f32(10 ** rng.uniform(-3, 3))
            tMin = f32(0.0 if rng.random() < 0.2 else 10 ** rng.uniform(-4, 6))
            # segment length in units of the mean free path, up to past the A < 40 cut
            A_target = 10 ** rng.uniform(-5, np.log10(45))
            segMax = f32(tMin + f32(A_target / sm0))
            if not segMax > tMin:
                continue
            dt = float(segMax) - float(tMin)
            # u near the boundary 1 - u = exp(-sm0 dt): within 1e-3 relative, or anywhere
            if rng.random() < 0.8:
                q = np.exp(-float(sm0) * dt) * (1 + rng.uniform(-3e-3, 3e-3))
                u = f32(min(max(1 - q, 0.0), 1 - 2 ** -24))
            else:
                u = f32(rng.random())
            n_checked += 1
            if _fast_reject(u, sm0, tMin, segMax):
                n_fast += 1
                assert _exact_reject(u, sm0, tMin, segMax), (float(u), float(sm0), float(tMin), float(segMax))
    finally:
        binding.set_libm("platform")
    # the sweep exercises the shortcut (not vacuous) and leaves the near-boundary cases pending
    assert n_fast > 0.2 * n_checked and n_fast < n_checked


def test_fast_reject_margin_covers_the_fastexp_error():
    """FastExp's relative error (< 3e-4 pinned by math_test.cpp:365-378; < 1.2e-4 observed for
    A < 40) stays inside the 1e-3 margin of the bound on a dense grid of A."""
    A = np.linspace(0.0, 40.0, 200001, dtype=np.float32)
    fe = np.array([binding.lib().oracle_fastexp(float(-a)) for a in A[::50]], np.float64)
    rel = np.abs(fe / np.exp(-A[::50].astype(np.float64)) - 1)
    assert rel.max() < 1.2e-4
