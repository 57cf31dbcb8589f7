"""render_row's byte-parallel decode (csrc/mgx_engine.hip: swar_type / swar_colour / swar_state and the dword
windows of the row assembly), restated on the host: for every cell code the grid can hold (types from
csrc/mgx_device.h, colours 0-5, the aux bit) the three planes equal the scalar decode render_cols applies, and a
row assembled from code dwords the way the kernel's four threads do is [direction][type 49][colour 49][state 49].
The GPU tests compare the kernel's rows with the oracle; this pins the arithmetic the kernel relies on (no cell
code 0 when see_through_walls=True; 11 is the only type with (t & 0b1011) == 0b1011, 4 the only one with
(t & 0b1011) == 0)."""
import os
import random
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _types():
    src = open(os.path.join(ROOT, "minigrid-rl_amd", "csrc", "mgx_device.h")).read()
    m = re.search(r"constexpr int (T_EMPTY = .*?);", src, re.S)
    return {k: int(v) for k, v in re.findall(r"(T_\w+) = (\d+)", m.group(1))}


def _scalar(v, T):
    t = v & 15
    return (T["T_DOOR"] if t == T["T_OPEN"] else t, (v >> 4) & 7, (1 + (v >> 7)) if t == T["T_DOOR"] else 0)


def _swar(w):
    t = w & 0x0F0F0F0F
    m = ((w & 0x0B0B0B0B) + 0x05050505) & 0x10101010
    ty = t ^ (m - (m >> 4))
    co = (w >> 4) & 0x07070707
    door = ((((w & 0x0B0B0B0B) + 0x0F0F0F0F) & 0x10101010) ^ 0x10101010) >> 4
    return ty & 0xFFFFFFFF, co, door + ((w >> 7) & door)


def _align(hi, lo, s):
    return (((hi << 32) | lo) >> (8 * s)) & 0xFFFFFFFF


def test_swar_planes_match_the_scalar_decode():
    T = _types()
    codes = [t | (c << 4) | (a << 7) for t in T.values() for c in range(6) for a in (0, 1)]
    rnd = random.Random(7)
    for _ in range(20000):
        b = [rnd.choice(codes) for _ in range(4)]
        planes = _swar(b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24)
        for i in range(4):
            assert tuple((p >> (8 * i)) & 255 for p in planes) == _scalar(b[i], T)


def test_row_assembly_from_code_windows():
    T = _types()
    codes = [t | (c << 4) | (a << 7) for t in T.values() for c in range(6) for a in (0, 1)]
    rnd = random.Random(11)
    for _ in range(300):
        cell = [rnd.choice(codes) for _ in range(49)]
        d = rnd.randrange(4)
        row = bytearray(rnd.randrange(256) for _ in range(148))
        row[4:53] = bytes(cell)                                   # pass 1: codes at row bytes 4 + c
        rw = [int.from_bytes(row[4 * k:4 * k + 4], "little") for k in range(37)]
        out = {}
        for q in range(4):                                        # pass 2, thread q
            c = [rw[q + 4 * j + i] for j in range(4) for i in range(2)]
            ty = [_swar(_align(c[2 * j + 1], c[2 * j], 3))[0] for j in range(3)]
            co = [_swar(_align(c[2 * j + 1], c[2 * j], 2))[1] for j in range(3)]
            st = [_swar(_align(c[2 * j + 1], c[2 * j], 1))[2] for j in range(4)]
            if q == 0:
                ty[0] = (ty[0] & 0xFFFFFF00) | d
                co[0] = (co[0] & 0xFFFF0000) | (_swar(_align(c[7], c[6], 3))[0] & 0xFFFF)
                st[0] = (st[0] & 0xFF000000) | (_swar(_align(c[7], c[6], 2))[1] & 0x00FFFFFF)
            for j in range(3):
                out[q + 4 * j], out[12 + q + 4 * j], out[24 + q + 4 * j] = ty[j], co[j], st[j]
            if q == 0:
                out[36] = st[3]
        assert sorted(out) == list(range(37))
        got = b"".join(out[k].to_bytes(4, "little") for k in range(37))
        dec = [_scalar(v, T) for v in cell]
        assert got == bytes([d] + [x[0] for x in dec] + [x[1] for x in dec] + [x[2] for x in dec])
