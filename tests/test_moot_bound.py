"""The moot shadow-ray test of the bounce setup (pt_wf.h wf_setup_core,
WF_SKIP_MOOT), restated in numpy float32 and checked against its claim: where
the test says "moot", each of the four occlusion outcomes of the light and env
shadow rays gives the shade's MIS sum (ray_tracing.comp:936-940, oracle
pn_oracle.c PathTracing "MIS") exactly Lo's bits -- so not tracing the rays
cannot change the image.

The restatement uses the kernel's operations in the kernel's order.  The
kernel's v_rcp_f32 is accurate to 1 ulp; the test takes the correctly rounded
quotient one ulp DOWN (the worst case for an upper bound).  Inputs: magnitudes
over the whole float range, zeros of both signs, negative pdfs (a BRDF sample
below the horizon gives dPDF < 0), infinities and NaNs, subnormals.  No GPU."""
import numpy as np
import pytest

F = np.float32


def _combos(Lo, cw, LD, pl, LE, pe, dPDF):
    """The shade's MIS sum for the four (light, env) outcomes (unoccluded or not)."""
    out = []
    with np.errstate(all="ignore"):
        for lu in (True, False):
            for eu in (True, False):
                ld = LD if lu else np.zeros_like(LD)
                plp = pl if lu else np.zeros_like(pl)
                le = LE if eu else np.zeros_like(LE)
                inv = F(1.0) / ((pe + plp) + dPDF)
                mis = le * pe[:, None] + ld * plp[:, None]
                out.append(Lo + (cw * mis) * inv[:, None])
    return out


def _moot(Lo, cw, LD, pl, LE, pe, dPDF, tsum=True):
    """pt_wf.h's test: T = (|cw| (|LE| pe + |LD| pl)) rU + (|cw| |LE| pe) rE
    (WF_MOOT_TSUM 1; 0: (|cw| (|LE| pe + |LD| pl)) max(rU, rE), fmaxf dropping a
    NaN quotient), rU / rE = rcp |(pe + pl) + dPDF| / |(pe + 0) + dPDF| times
    (1 + 2^-20); moot where Lo + T == Lo and Lo - T == Lo in every channel."""
    with np.errstate(all="ignore"):
        acw = np.abs(cw)
        mE = np.abs(LE) * np.abs(pe)[:, None]
        mU = mE + np.abs(LD) * np.abs(pl)[:, None]

        def rcp_low(d):     # v_rcp_f32 within 1 ulp: the quotient one ulp toward zero; a
            q = F(1.0) / np.abs(d)          # subnormal result may come back flushed to 0
            return np.where(q < F(2.0 ** -126), F(0.0), np.nextafter(q, F(0.0))).astype(F)

        rU = rcp_low((pe + pl) + dPDF) * (F(1.0) + F(2.0 ** -20))
        rE = rcp_low((pe + F(0.0)) + dPDF) * (F(1.0) + F(2.0 ** -20))
        if tsum:
            T = (acw * mU) * rU[:, None] + (acw * mE) * rE[:, None]
        else:
            T = (acw * mU) * np.fmax(rU, rE)[:, None]
        hi, lo = Lo + T, Lo - T
        ok = (rU >= F(2.0 ** -126)) & (rE >= F(2.0 ** -126))
        return ok & np.all((hi == Lo) & (lo == Lo), axis=1)


def _draw(rng, n, shape=()):
    """Floats across the range: log-uniform magnitudes, random signs, and a share
    of specials (0, -0, inf, nan, subnormal)."""
    mag = F(2.0) ** rng.uniform(-140, 120, size=(n,) + shape).astype(F)
    v = (mag * rng.choice([F(1), F(-1)], size=(n,) + shape, p=[0.8, 0.2])).astype(F)
    sp = rng.random((n,) + shape)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-42, 3e-39], F)
    v = np.where(sp < 0.08, specials[rng.integers(0, len(specials), (n,) + shape)], v)
    return v.astype(F)




@pytest.mark.parametrize("tsum", [True, False])
def test_moot_implies_every_outcome_equal(tsum):
    rng = np.random.default_rng(11)
    hits = 0
    for _ in range(10):
        n = 200_000
        Lo = np.abs(_draw(rng, n, (3,)))      # Lo >= +0 (never -0): sums of the path's terms from +0
        Lo = np.where(rng.random((n, 3)) < 0.5, (Lo * F(1e-30)).astype(F), Lo)
        cw, LD, LE = _draw(rng, n, (3,)), _draw(rng, n, (3,)), _draw(rng, n, (3,))
        # realistic-range rows too, where the absorption case is common
        real = rng.random(n) < 0.5
        Lo[real] = rng.uniform(0.01, 2.0, (real.sum(), 3)).astype(F)
        cw[real] = (rng.uniform(0, 1, (real.sum(), 3)) ** 8).astype(F)
        LD[real] = (rng.uniform(0, 1, (real.sum(), 3)) * F(2.0) ** rng.uniform(-50, 5, (real.sum(), 1))).astype(F)
        LE[real] = (rng.uniform(0, 1, (real.sum(), 3)) * F(2.0) ** rng.uniform(-50, 5, (real.sum(), 1))).astype(F)
        pl, pe, dPDF = _draw(rng, n), np.abs(_draw(rng, n)), _draw(rng, n)
        pl[real] = F(2.0) ** rng.uniform(-5, 30, real.sum()).astype(F)
        pe[real] = rng.uniform(0, 3, real.sum()).astype(F)
        dPDF[real] = rng.uniform(-0.5, 3, real.sum()).astype(F)
        m = _moot(Lo, cw, LD, pl, LE, pe, dPDF, tsum)
        hits += int(m.sum())
        for c in _combos(Lo, cw, LD, pl, LE, pe, dPDF):
            bad = m & ~np.all(c.view(np.uint32) == Lo.view(np.uint32), axis=1)
            assert not bad.any(), (Lo[bad][:3], cw[bad][:3], LD[bad][:3], pl[bad][:3], LE[bad][:3], pe[bad][:3],
                                   dPDF[bad][:3])
    assert hits > 50_000         # the test does fire (absorbed terms, zero weights)


def test_moot_edge_cases():
    """Hand-picked rows: an exactly zero path weight with a negative or zero pdf
    sum (moot only while the quotient is finite), a NaN / inf operand (never
    moot), a term just above / below Lo's rounding."""
    one = np.ones((1, 3), F)
    cases = [
        # Lo, cw, LD, pl, LE, pe, dPDF, expected
        (one * 0.3, one * 0.0, one * 0.5, 17.0, one * 0.0, 0.0, -0.9, True),
        (one * 0.3, one * 0.0, one * 0.5, 0.9, one * 0.0, 0.0, -0.9, False),    # 0.9 - 0.9 = 0: 1/0 = inf
        (one * 0.3, one * 0.0, one * np.nan, 1.0, one * 0.0, 0.0, 1.0, False),
        (one * 0.3, one * 0.0, one * np.inf, 1.0, one * 0.0, 0.0, 1.0, False),
        (one * 1.0, one * 1.0, one * 2.0 ** -30, 1.0, one * 0.0, 0.0, 1.0, True),
        (one * 1.0, one * 1.0, one * 2.0 ** -20, 1.0, one * 0.0, 0.0, 1.0, False),
        (one * 0.0, one * 1.0, one * 0.0, 3.0, one * 0.0, 0.0, 0.5, True),       # dark light, no env term
        (one * 0.0, one * 1.0, one * 0.0, 3.0, one * 1e-30, 0.2, 0.5, False),
        # a denominator above 2^126: the reciprocal may flush to 0 and bound nothing
        (one * 0.0, one * 1.0, one * 1.0, 1e38, one * 0.0, 0.0, 0.5, False),
        (one * 0.0, one * 0.5, one * 0.0, 1.0, one * 0.0, 0.0, 3e38, False),
    ]
    for Lo, cw, LD, pl, LE, pe, dPDF, want in cases:
        args = [np.asarray(v, F) for v in (Lo, cw, LD)] + [np.array([pl], F)] + [np.asarray(LE, F)] + \
            [np.array([pe], F), np.array([dPDF], F)]
        got = bool(_moot(*args)[0])
        assert got == want, (Lo, cw, LD, pl, LE, pe, dPDF)
        if got:
            for c in _combos(*args):
                assert np.array_equal(c.view(np.uint32), args[0].view(np.uint32))


def _cont_moot(Lo, cw, E, dBRDF, NdotL, dPDF, mis_same):
    """pt_wf.h's last-bounce continuation test: Tc = ((|cw| E) |dBRDF|) NdotL
    rcp(|dPDF|) (1 + 2^-20); moot where Tc == 0, or where the MIS test held and
    Lo +- Tc round to Lo."""
    with np.errstate(all="ignore"):
        q = F(1.0) / np.abs(dPDF)
        rc = np.where(q < F(2.0 ** -126), F(0.0), np.nextafter(q, F(0.0))).astype(F) * (F(1.0) + F(2.0 ** -20))
        Tc = (((np.abs(cw) * E[:, None]) * np.abs(dBRDF)) * NdotL[:, None]) * rc[:, None]
        zero = np.all(Tc == 0, axis=1)
        near = np.all((Lo + Tc == Lo) & (Lo - Tc == Lo), axis=1)
        return (rc >= F(2.0 ** -126)) & (zero | (mis_same & near))


def test_last_bounce_continuation_moot():
    """Where the continuation test says moot, the term the last bounce's hit or
    miss adds -- (((cw em) dBRDF) NdotL) / dPDF (ray_tracing.comp:950-969), for
    any em with |em| <= E -- leaves Lo1's bits (Lo1 = Lo where the MIS test held,
    any value but -0 otherwise)."""
    rng = np.random.default_rng(12)
    hits = zeros = 0
    for _ in range(10):
        n = 200_000
        Lo = np.abs(_draw(rng, n, (3,)))
        cw, dBRDF = _draw(rng, n, (3,)), _draw(rng, n, (3,))
        E = np.abs(_draw(rng, n))
        NdotL = np.abs(_draw(rng, n))
        dPDF = _draw(rng, n)
        real = rng.random(n) < 0.6
        k = int(real.sum())
        Lo[real] = rng.uniform(0.01, 2.0, (k, 3)).astype(F)
        cw[real] = np.where(rng.random((k, 3)) < 0.3, F(0), (rng.uniform(0, 1, (k, 3)) ** 12)).astype(F)
        dBRDF[real] = np.where(rng.random((k, 1)) < 0.3, F(0), rng.uniform(0, 1, (k, 3))).astype(F)
        E[real] = rng.uniform(0, 50, k).astype(F)
        NdotL[real] = rng.uniform(0, 1, k).astype(F)
        dPDF[real] = rng.uniform(-0.5, 3, k).astype(F)
        mis_same = rng.random(n) < 0.5
        m = _cont_moot(Lo, cw, E, dBRDF, NdotL, dPDF, mis_same)
        hits += int(m.sum())
        zeros += int((m & ~mis_same).sum())
        for trial in range(4):
            sign = rng.choice([F(1), F(-1)], size=(n, 3))
            frac = [F(1), F(0), rng.uniform(0, 1, (n, 3)).astype(F), F(2.0 ** -30)][trial]
            with np.errstate(all="ignore"):
                em = (E[:, None] * frac * sign).astype(F)      # (inf * 0: NaN emission rows test NaN too)
                term = (((cw * em) * dBRDF) * NdotL[:, None]) / dPDF[:, None]
                # the MIS test held: Lo1 = Lo; otherwise Lo1 is any value but -0
                Lo1 = np.where(mis_same[:, None], Lo, np.abs(_draw(rng, n, (3,))))
                out = Lo1 + term
            bad = m & ~np.all(out.view(np.uint32) == Lo1.view(np.uint32), axis=1)
            assert not bad.any(), (Lo1[bad][:2], cw[bad][:2], E[bad][:2], dBRDF[bad][:2], NdotL[bad][:2], dPDF[bad][:2])
    assert hits > 100_000 and zeros > 10_000
