#!/usr/bin/env python3
"""Regenerates tests/golden/golden_{8,10}.npz — TEST INFRASTRUCTURE.

The reference publishes no golden vectors for this path and its C path is not
buildable here, so these fixtures freeze the outputs of the
oracle (oracle/oracle.c) on the reference's own checkasm inputs (glibc rand,
seed 12345, tools/checkasm.c) and on small synthetic frames.  Every value is
cross-checked against the independent numpy restatement before it is written.
Inputs are not stored; their SHA-256 is, so a drift of the input generators is
caught separately from a drift of the kernels.

usage: python tests/golden/make_golden.py
"""
import hashlib
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
ROOT = os.path.dirname(TESTS)
sys.path.insert(0, TESTS)

import checkasm_bufs as cb  # noqa: E402
import numpy_ref as nr  # noqa: E402
import oracle_lib as orc  # noqa: E402


def synth_module():
    spec = importlib.util.spec_from_file_location("synth", os.path.join(ROOT, "x264-i386pic_amd", "synth.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


OPS = ("sad", "ssd", "satd")
NPOPS = {"sad": nr.sad, "ssd": nr.ssd, "satd": nr.satd}
DCT_SHAPES = {"sub4x4_dct": (4, 4), "sub8x8_dct": (8, 8), "sub16x16_dct": (16, 16), "sub8x8_dct_dc": (8, 8),
              "sub8x16_dct_dc": (8, 16), "sub8x8_dct8": (8, 8), "sub16x16_dct8": (16, 16)}
NPDCT = {"sub4x4_dct": nr.sub4x4_dct, "sub8x8_dct": nr.sub8x8_dct, "sub16x16_dct": nr.sub16x16_dct,
         "sub8x8_dct_dc": nr.sub8x8_dct_dc, "sub8x16_dct_dc": nr.sub8x16_dct_dc, "sub8x8_dct8": nr.sub8x8_dct8,
         "sub16x16_dct8": nr.sub16x16_dct8}
QPS = (0, 6, 12, 20, 26, 33, 40, 47, 51)


def compute(bd):
    """All fixture arrays for one bit depth (inputs regenerated deterministically)."""
    out = {}
    b = cb.Bufs(bd)
    b.fill_pixel_overflow()
    out["in_sha_pixel"] = np.frombuffer(sha(b.pbuf1, b.pbuf3, b.pbuf4).encode(), np.uint8)
    pix = np.zeros((3, 8, 80), np.int32)
    for k, op in enumerate(OPS):
        for i, (w, h) in enumerate(nr.SIZES):
            for j in range(64):
                s1 = 32 if (j & 31) == 31 else 16
                v = orc.cmp(bd, op, i, b.pbuf1, 0, s1, b.pbuf1, b.pbuf2_off + j, 64)
                assert v == NPOPS[op](nr.block(b.pbuf1, 0, s1, w, h), nr.block(b.pbuf1, b.pbuf2_off + j, 64, w, h))
                pix[k, i, j] = v
            for t, j in enumerate(range(0, 0x1000, 256)):
                v = orc.cmp(bd, op, i, b.pbuf3, j, 16, b.pbuf4, j, 16)
                assert v == NPOPS[op](nr.block(b.pbuf3, j, 16, w, h), nr.block(b.pbuf4, j, 16, w, h))
                pix[k, i, 64 + t] = v
    out["pixel"] = pix
    x4 = np.zeros((2, 7, 64, 4), np.int32)
    for k, op in enumerate(("sad", "satd")):
        for i in range(7):
            for j in range(64):
                base = b.pbuf2_off + j
                x4[k, i, j] = orc.cmp_x(bd, op, 4, i, b.pbuf1, 0, b.pbuf1, [base, base + 6, base + 1, base + 10], 64)
    out["pixel_x4"] = x4

    b = cb.Bufs(bd)
    b.fill_dct_overflow()
    out["in_sha_dct"] = np.frombuffer(sha(b.pbuf1, b.pbuf3, b.pbuf4).encode(), np.uint8)
    for name, (w, h) in DCT_SHAPES.items():
        res = []
        for j in range(5):
            for (a, ao, d, do) in ((b.pbuf1, j * 64, b.pbuf1, b.pbuf2_off + j * 64),
                                   (b.pbuf3, 16 * j * 16, b.pbuf4, 16 * j * 32)):
                v = orc.sub_dct(bd, name, a, ao, d, do)
                want = NPDCT[name](nr.block(a, ao, 16, w, h) - nr.block(d, do, 32, w, h), bd)
                assert np.array_equal(v.astype(np.int64), want.ravel())
                res.append(v)
        out["dct_" + name] = np.stack(res)

    cb.srand(cb.SEED)
    cqm_all, quant_all = [], []
    for i_cqm in range(6):
        lists = cb.cqm_lists(i_cqm, bd)
        tabs = orc.cqm_init(bd, lists)
        for g, w in zip(tabs, nr.cqm_init(bd, lists)):
            assert np.array_equal(g, w)
        cqm_all.append(np.concatenate([t.ravel().astype(np.int64) for t in tabs]))
        q4m, q4b, q8m, q8b = tabs
        for qp in QPS:
            qp = min(qp + 6 * (bd - 8) if qp == 51 else qp, 51 + 6 * (bd - 8))
            c8 = cb.init_quant8(1, bd)
            c4 = cb.init_quant4(1, 16, bd)
            v8, n8 = orc.quant(bd, "quant_8x8", c8, q8m[1, qp], q8b[1, qp])
            v4, n4 = orc.quant(bd, "quant_4x4", c4, q4m[1, qp], q4b[1, qp])
            assert np.array_equal(v8, nr.quant(c8, q8m[1, qp], q8b[1, qp], bd)[0])
            assert np.array_equal(v4, nr.quant(c4, q4m[1, qp], q4b[1, qp], bd)[0])
            quant_all.append(np.concatenate([c8, v8.astype(np.int64), [n8], c4, v4.astype(np.int64), [n4]]))
    out["cqm"] = np.stack(cqm_all)
    out["quant"] = np.stack(quant_all)

    synth = synth_module()
    planes, stride, origin = synth.make_sequence(2, 64, 48, bd)
    out["in_sha_frames"] = np.frombuffer(sha(planes).encode(), np.uint8)
    out["me_full_r8"] = orc.me_search_full(bd, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride,
                                           4, 3, 8)
    q4m, q4b, q8m, q8b = orc.cqm_init(bd, [cb.FLAT16] * 8)
    qp = 26 + 6 * (bd - 8)
    d4, n4 = orc.mb_dct_quant(bd, 4, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, 4, 3,
                              q4m[1, qp], q4b[1, qp])
    d8, n8 = orc.mb_dct_quant(bd, 8, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, 4, 3,
                              q8m[1, qp], q8b[1, qp])
    out["mb_dct4_quant"], out["mb_dct4_nz"] = d4, n4
    out["mb_dct8_quant"], out["mb_dct8_nz"] = d8, n8
    out.update(compute_ext(bd, planes, stride, origin, d4, d8))
    return out


def compute_ext(bd, planes, stride, origin, d4, d8):
    """Fixtures of the further pixel entries, the inverse path and the lookahead /
    motion-compensation inputs (§8f), cross-checked against numpy where a
    restatement exists (tests/test_cpu_pixel_ext.py, test_cpu_inverse.py)."""
    out = {}
    b = cb.Bufs(bd)
    b.fill_pixel_overflow()
    p1 = b.pbuf1
    # sa8d / sa8d_satd (TEST_PIXEL inputs), hadamard_ac, var, var2
    sa = np.zeros((2, 80), np.int64)
    ss = np.zeros(80, np.uint64)
    for k, i in enumerate((0, 3)):
        w, h = nr.SIZES[i]
        for j in range(64):
            s1 = 32 if (j & 31) == 31 else 16
            sa[k, j] = orc.sa8d(bd, i, p1, 0, s1, p1, b.pbuf2_off + j, 64)
            assert sa[k, j] == nr.sa8d(nr.block(p1, 0, s1, w, h), nr.block(p1, b.pbuf2_off + j, 64, w, h))
        for t, j in enumerate(range(0, 0x1000, 256)):
            sa[k, 64 + t] = orc.sa8d(bd, i, b.pbuf3, j, 16, b.pbuf4, j, 16)
    for j in range(64):
        ss[j] = orc.sa8d_satd(bd, p1, 0, 16, p1, b.pbuf2_off + j, 64)
    for t, j in enumerate(range(0, 0x1000, 256)):
        ss[64 + t] = orc.sa8d_satd(bd, b.pbuf3, j, 16, b.pbuf4, j, 16)
    out["sa8d"], out["sa8d_satd"] = sa, ss
    hac = np.zeros((4, 32), np.uint64)
    for i in range(4):
        w, h = nr.SIZES[i]
        for j in range(32):
            buf = p1 if j & 16 else b.pbuf3
            off = (j & 15) * 256
            if off + 16 * (h - 1) + w <= buf.size:
                hac[i, j] = orc.hadamard_ac(bd, i, buf, off, 16)
                assert hac[i, j] == nr.hadamard_ac(nr.block(buf, off, 16, w, h))
    out["hadamard_ac"] = hac
    out["var"] = np.array([[orc.var(bd, i, buf, off, 16) for buf, off in ((p1, 0), (p1, 77), (b.pbuf3, 256))]
                           for i in (0, 2, 3)], np.uint64)
    out["var2"] = np.array([orc.var2(bd, i, p1, fo, p1, do) for i in (2, 3)
                            for fo, do in ((0, b.pbuf2_off), (64, b.pbuf2_off + 5))], np.int64)
    # ads over the checkasm distributions (glibc rand, seed 4321)
    pm = (1 << bd) - 1
    cb.srand(4321)
    cost = np.array([cb.rand30() & 0xFFFF for _ in range(32)], np.uint16)
    ads = np.full((100, 29), -1, np.int16)
    for i in range(100):
        ns = (4, 2, 2, 1)[i & 3]
        thresh = (cb.rand() % 257) * pm + (cb.rand30() & 0xFFFF)
        if i < 40:
            sums = np.array([(cb.rand() % 9) * 8 * pm for _ in range(72)], np.int64).astype(np.uint16)
            dc = np.array([(cb.rand() % 9) * 8 * pm for _ in range(4)], np.int32)
        else:
            r = cb.rand30 if bd + 6 > 15 else cb.rand
            sums = np.array([r() & ((1 << (bd + 6)) - 1) for _ in range(72)], np.uint16)
            dc = np.array([r() & ((1 << (bd + 6)) - 1) for _ in range(4)], np.int32)
        mv = orc.ads(bd, ns, dc, sums, 0, 32, cost, 0, 28, thresh)
        ads[i, 0] = len(mv)
        ads[i, 1:1 + len(mv)] = mv
    out["ads"] = ads
    # inverse path on the forward fixtures above: dequant at qp 26 (flat lists) and
    # reconstruction of the 64x48 pair; coefficient statistics / scans of the MB coefs
    dq4, dq8 = orc.cqm_dequant([cb.FLAT16] * 8)
    qp = 26 + 6 * (bd - 8)
    nmb = d4.shape[0]
    qpm = np.full(nmb, qp, np.int32)
    for t, d, dq in ((4, d4, dq4[1]), (8, d8, dq8[1])):
        rec = np.zeros_like(planes[0]).ravel()
        orc.mb_dequant_idct_add(bd, t, d, 4, 3, dq, qpm, planes[0].ravel(), origin, stride, rec, origin, stride)
        out[f"recon{t}"] = rec.reshape(planes[0].shape)[32:32 + 48, 32:32 + 64].copy()
    blocks = d4.reshape(-1, 16)
    out["decimate16"] = np.array([orc.inplace(bd, "decimate_score16", x)[1] for x in blocks], np.int32)
    out["coeff_last16"] = np.array([orc.fn(bd, "coeff_last")(orc._addr(np.ascontiguousarray(x)), 16) for x in blocks],
                                   np.int32)
    out["zigzag4_frame"] = np.stack([orc.zigzag_scan(bd, 16, 0, x) for x in blocks])
    out["zigzag8_field"] = np.stack([orc.zigzag_scan(bd, 64, 1, x) for x in d8.reshape(-1, 64)])
    rs = np.random.default_rng(99)
    c16 = rs.integers(-(1 << (bd + 1)), 1 << (bd + 1), (12, 16))
    out["dequant4"] = np.stack([orc.inplace(bd, "dequant_4x4", c16[q % 12], orc._addr(dq4[0]), q)[0]
                                for q in range(0, 52 + 6 * (bd - 8), 4)])
    # motion-compensation / lookahead inputs on the same synthetic frame
    hp = orc.frame_filter(bd, planes[0].ravel().copy(), origin, stride, 64, 48)
    out["hpel"] = np.stack([x.reshape(planes[0].shape) for x in hp])
    ls = (32 + 64 + 63) // 64 * 64
    out["lowres"] = np.stack(orc.frame_init_lowres(bd, planes[0].ravel(), origin, stride, 64, 48, ls))
    integ = orc.frame_integral(bd, planes[0].ravel(), origin, stride, 48, 32, 1)
    out["integral"] = integ
    box = nr.box_sums(planes[0].astype(np.int64), 8)
    assert np.array_equal(integ[1:48 + 56, :stride - 8], box[1:48 + 56, :stride - 8])
    return out


def main():
    for bd in (8, 10):
        arrays = compute(bd)
        path = os.path.join(HERE, f"golden_{bd}.npz")
        np.savez_compressed(path, **arrays)
        print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
