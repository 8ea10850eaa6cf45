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


def _spectrum_scale(beta, n, fmin=0.0):
    f = np.fft.rfftfreq(n)
    fmin = max(fmin, 1.0 / n)
    scale = f.copy()
    cut = np.sum(scale < fmin)
    if cut < scale.size:
        scale[:cut] = scale[cut]
    scale = scale ** (-beta / 2.0)
    w = scale[1:].copy()
    w[-1] *= (1 + (n % 2)) / 2.0
    return scale, 2 * np.sqrt(np.sum(w ** 2)) / n


def powerlaw_psd_gaussian_device(beta, rows, n, device, generator=None, spectrum=None):
    """The same power-law noise generated on the GPU (torch.randn + hipFFT
    irfft), one independent sequence of length n per row: [rows, n] float32.
    `spectrum` = (sr, si) [rows, n//2+1] replaces the Gaussian draws (tests)."""
    import torch
    scale, sigma = _spectrum_scale(beta, n)
    nf = scale.size
    sc = torch.as_tensor(scale, dtype=torch.float64, device=device)
    if spectrum is None:
        sr = torch.randn((rows, nf), dtype=torch.float64, device=device, generator=generator) * sc
        si = torch.randn((rows, nf), dtype=torch.float64, device=device, generator=generator) * sc
    else:
        sr, si = (torch.as_tensor(x, dtype=torch.float64, device=device).clone() for x in spectrum)
    if n % 2 == 0:
        si[..., -1] = 0
        sr[..., -1] *= np.sqrt(2)
    si[..., 0] = 0
    sr[..., 0] *= np.sqrt(2)
    return (torch.fft.irfft(torch.complex(sr, si), n=n, dim=-1) / sigma).float()


def irfft_reference(sr, si, beta, n):
    """numpy path of the deterministic half (for tests): the same masking and
    normalisation as powerlaw_psd_gaussian applied to given spectra."""
    _, sigma = _spectrum_scale(beta, n)
    sr, si = np.array(sr, dtype=np.float64), np.array(si, dtype=np.float64)
    if n % 2 == 0:
        si[..., -1] = 0
        sr[..., -1] *= np.sqrt(2)
    si[..., 0] = 0
    sr[..., 0] *= np.sqrt(2)
    return np.fft.irfft(sr + 1j * si, n=n, axis=-1) / sigma
