"""CPU model of sed_ck_codes_kernel's code re-layout (sed_kernels.hip, config 2's checkpoint route).

A tile's sweep leaves lane r (= 4b + rr: forward lane 16Q + b, row rr) with the codes of sweep steps 0..127 in W[8]
(step sigma at W[sigma >> 4] bits 2 (sigma & 15)).  The kernel takes each lane's 64 codes from sweep step
15 + 3b + rr on (one funnel shift), and lane 4b' + g interleaves rows 4b'..4b'+3 of window word g into the store_tb
layout of forward lane 16Q + b', group 4c + g: word w holds steps u = 4w..4w+3, code (u, rr) at bits 2 (4u + rr) of
the group.  This restates that index arithmetic on random codes and checks it against the layout's definition: the
code of row rr of forward lane t at forward step s = 64c + 16g + u is the sweep code of lane 4b + rr at step
s - 64c + 15 + 3b + rr.  (The GPU test of the route is tests/test_gpu_routes.py::test_split_checkpoint_codes_route.)"""
import numpy as np

R, G = 4, 16


def transpose4x4(y):
    t = ((y >> 6) ^ y) & 0x00CC00CC
    y ^= t ^ ((t << 6) & 0xFFFFFFFF)
    t = ((y >> 12) ^ y) & 0x0000F0F0
    return (y ^ t ^ ((t << 12) & 0xFFFFFFFF)) & 0xFFFFFFFF


def perm(a, b, sel):
    """v_perm_b32: bytes of {a (bytes 4..7), b (bytes 0..3)}; selector 0x0C = zero."""
    src = [(b >> (8 * i)) & 0xFF for i in range(4)] + [(a >> (8 * i)) & 0xFF for i in range(4)]
    out = 0
    for i in range(4):
        k = (sel >> (8 * i)) & 0xFF
        out |= (src[k] if k < 8 else 0) << (8 * i)
    return out


def kernel_model(W):
    """W: 64 lanes x 8 words.  Returns {(b', g): [o0, o1, o2, o3]} as sed_ck_codes_kernel writes them."""
    win = {}
    for lane in range(64):
        b, rr = lane >> 2, lane & 3
        s0 = G - 1 + (R - 1) * b + rr
        x = [int(W[lane][(s0 >> 4) + i]) for i in range(5)]
        sh = (2 * s0) & 31
        win[lane] = [((x[i] >> sh) | (x[i + 1] << (32 - sh))) & 0xFFFFFFFF if sh else x[i] for i in range(4)]
    out = {}
    for lane in range(64):
        bo, g = lane >> 2, lane & 3
        y = [win[4 * bo + q][g] for q in range(4)]
        o = []
        for w in range(4):
            sel = (w * 0x0101 + 0x0400) | 0x0C0C0000
            y01, y23 = perm(y[1], y[0], sel), perm(y[3], y[2], sel)
            o.append(transpose4x4(perm(y23, y01, 0x05040100)))
        out[(bo, g)] = o
    return out


def test_code_relayout_matches_the_store_tb_layout():
    rng = np.random.default_rng(7)
    for _ in range(5):
        codes = rng.integers(0, 3, size=(64, 128))  # sweep code of lane r at step sigma
        W = [[sum(int(codes[r][16 * w + i]) << (2 * i) for i in range(16)) for w in range(8)] for r in range(64)]
        out = kernel_model(W)
        for (bo, g), words in out.items():
            for u in range(16):  # forward step 64c + 16g + u
                for rr in range(4):
                    c = u * R + rr
                    got = (words[c >> 4] >> (2 * (c & 15))) & 3
                    sigma = (16 * g + u) + G - 1 + (R - 1) * bo + rr
                    assert got == codes[4 * bo + rr][sigma]
