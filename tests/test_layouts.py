"""Host-side checks of the LDS / slab layouts the training kernel relies on (restated from
neural-radiance-caching_amd/csrc/nrc_kernels.hip img_off / tr_frag and csrc/nrc_internal.h acc_row /
slab_block_base): the image layout is a bijection, pairs each lane's two 4-feature quads into one 16-byte slot,
and keeps both the 16-byte row writes and the transposed reads free of LDS bank conflicts
(MI355X_MICROARCH.md §LDS bank rules: ds_write_b128 in 8-lane groups over 32 banks, ds_read_b64_tr_b16 in
32-lane halves over 64 banks)."""


def acc_row(kk, h, j):
    return 32 * (kk >> 1) + 16 * (kk & 1) + 8 * (j >> 2) + 4 * h + (j & 3)


def img_off(s, c):
    lq = c >> 2
    pq = (lq & ~3) | ((lq & 1) << 1) | ((lq >> 1) & 1)
    hs = (s & 1) | (((s >> 2) & 1) << 1) | (((s >> 1) & 1) << 2)
    return s * 128 + (((pq >> 1) ^ hs) << 4) + ((pq & 1) << 3) + ((c & 3) << 1)


def test_image_is_a_bijection_with_16_byte_fragments():
    offs = {img_off(s, c) for s in range(128) for c in range(64)}
    assert len(offs) == 128 * 64 and max(offs) < 128 * 128 and min(offs) == 0
    for kk in range(4):
        for h in range(2):
            for s in range(128):
                base = img_off(s, acc_row(kk, h, 0))
                assert base % 16 == 0
                assert [img_off(s, acc_row(kk, h, j)) for j in range(8)] == [base + 2 * j for j in range(8)]


def test_row_writes_are_conflict_free():
    for kk in range(4):
        for h in range(2):
            for s0 in range(0, 128, 8):  # ds_write_b128: lanes (= samples) in groups of 8, banks (a/4) mod 32
                banks = [((img_off(s, acc_row(kk, h, 0)) // 4) + i) % 32 for s in range(s0, s0 + 8) for i in range(4)]
                assert len(set(banks)) == 32


def test_transposed_reads_are_conflict_free():
    for fb in range(2):
        for kk in range(8):
            for second in range(2):
                for half in range(2):  # ds_read_b64_tr_b16: 32-lane halves, banks (a/4) mod 64
                    banks = []
                    for lane in range(32 * half, 32 * half + 32):
                        g, idx = lane >> 4, lane & 15
                        q, p = idx >> 2, idx & 3
                        c = 32 * fb + 16 * (g & 1) + 4 * p
                        s = 16 * kk + 8 * (g >> 1) + q + 4 * second
                        a = img_off(s, c)
                        banks += [((a // 4) + i) % 64 for i in range(2)]
                    assert len(set(banks)) == 64


def slab_block_base(enc, L, mb, nb):
    nb0 = 2 if enc == 1 else 3
    if L == 0:
        return (mb * nb0 + nb) * 1024
    if L <= 4:
        return 2 * nb0 * 1024 + (L - 1) * 4096 + (mb * 2 + nb) * 1024
    return 2 * nb0 * 1024 + 4 * 4096 + nb * 512


def test_slab_positions_cover_every_weight_once():
    """Fragment-major slab: every (layer, row, column) of dW lands on exactly one position."""
    for enc, in0, n in ((0, 80, 22528), (1, 64, 21504)):
        seen = {}
        for L in range(6):
            nmb, nnb, nreg = (1, 2, 8) if L == 5 else (2, 3 if (L == 0 and enc != 1) else 2, 16)
            for mb in range(nmb):
                for nb in range(nnb):
                    for lane in range(64):
                        for reg in range(nreg):
                            row = 32 * mb + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
                            col = 32 * nb + (lane & 31)
                            if L == 0 and col >= in0:
                                continue
                            pos = slab_block_base(enc, L, mb, nb) + ((reg >> 2) * 64 + lane) * 4 + (reg & 3)
                            key = (L, row, col)
                            assert key not in seen and pos not in seen.values()
                            seen[key] = pos
        assert len(seen) == n
        assert max(seen.values()) < slab_block_base(enc, 5, 0, 2)


# ---- t16 training layout (neural-radiance-caching_amd/csrc/nrc_train16.hip swz64 / off64 / swz32 / off32)
def swz64(r):
    return (r & 1) | (((r >> 2) & 1) << 1) | (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3)


def off64(r, Q):
    return r * 128 + 8 * (Q ^ swz64(r))


def swz32(r):
    return ((r >> 1) & 1) | (((r >> 2) & 1) << 1) | (((r >> 3) & 1) << 2)


def off32(r, Q):
    return r * 64 + 8 * (Q ^ swz32(r))


def test_t16_images_are_bijections():
    assert sorted(off64(r, Q) for r in range(128) for Q in range(16)) == list(range(0, 128 * 128, 8))
    assert sorted(off32(r, Q) for r in range(128) for Q in range(8)) == list(range(0, 128 * 64, 8))


def test_t16_row_writes_are_conflict_free():
    # ds_write_b64: 16 contiguous lanes per LDS cycle, banks (a / 4) mod 32; a 16-lane group is 16 consecutive
    # samples (rows 16k .. 16k + 15) writing the same quad
    for off, nq in ((off64, 16), (off32, 8)):
        for k in range(8):
            for Q in range(nq):
                banks = [(off(16 * k + c, Q) // 4 + i) % 32 for c in range(16) for i in range(2)]
                assert len(set(banks)) == 32, (off.__name__, k, Q)


def test_t16_transposed_reads_are_conflict_free():
    # ds_read_b64_tr_b16: 32-lane halves, banks (a / 4) mod 64; lane (G, q, p) reads row 32 kk + 8 G + q (+ 4) of the
    # tile's quad 4 t + p
    for off, ntile in ((off64, 4), (off32, 2)):
        for t in range(ntile):
            for kk in range(4):
                for second in range(2):
                    for half in range(2):
                        banks = []
                        for lane in range(32 * half, 32 * half + 32):
                            G, q, p = lane >> 4, (lane >> 2) & 3, lane & 3
                            a = off(32 * kk + 8 * G + 4 * second + q, 4 * t + p)
                            banks += [(a // 4) % 64, (a // 4 + 1) % 64]
                        assert len(set(banks)) == 64, (off.__name__, t, kk, second, half)


def test_t16_slot_and_slab_maps_host_check(tmp_path):
    """tests/cpp/t16_maps_check.cpp compiled for the host against csrc/nrc_internal.h: the t16 layer-0 slot maps
    (Frequency, Hash) put every canonical feature in exactly one K slot, the closed-form slab inverses reach every MLP
    parameter exactly once, and the Hash W0^T fragments do not collide (no GPU needed)."""
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "t16_maps_check"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", f"-I{root / 'include'}",
                        f"-I{root / 'neural-radiance-caching_amd' / 'csrc'}", str(root / "tests" / "cpp" / "t16_maps_check.cpp"),
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and "t16 maps OK" in out.stdout, out.stdout + out.stderr
