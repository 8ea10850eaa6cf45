"""Power-law ("coloured") Gaussian noise for per-episode exploration.

Used by select_action of Agent/TD7_multi_agent_Pink_noise.py:203-228 through
Agent/Pink_noise.py (ColoredActionNoise) and Agent/colorednoise.py.  This is an
independent implementation of the published algorithm those files implement
(J. Timmer and M. Koenig, "On generating power law noise", A&A 300, 1995):
draw a Gaussian spectrum with amplitude ~ f^(-beta/2), zero the imaginary parts
that must be real, inverse-FFT, and normalise to unit variance.
"""
import numpy as np


def powerlaw_psd_gaussian(beta, size, fmin=0.0, rng=None):
    rng = np.random.default_rng() if rng is None else rng
    size = (size,) if np.isscalar(size) else tuple(size)
    n = size[-1]
    f = np.fft.rfftfreq(n)
    fmin = max(fmin, 1.0 / n)
    scale = f.copy()
    cut = np.sum(scale < fmin)
    if cut < scale.size:
        scale[:cut] = scale[cut]
    scale = scale ** (-beta / 2.0)
    w = scale[1:].copy()
    w[-1] *= (1 + (n % 2)) / 2.0
    sigma = 2 * np.sqrt(np.sum(w ** 2)) / n
    shape = size[:-1] + (f.size,)
    sr = rng.normal(scale=scale, size=shape)
    si = rng.normal(scale=scale, size=shape)
    if n % 2 == 0:
        si[..., -1] = 0
        sr[..., -1] *= np.sqrt(2)
    si[..., 0] = 0
    sr[..., 0] *= np.sqrt(2)
    return np.fft.irfft(sr + 1j * si, n=n, axis=-1) / sigma
