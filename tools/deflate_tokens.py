"""Token statistics of a PNG's zlib stream (blocks, literals, matches by
distance class): what the serial one-wave inflate spends its symbols on.

    python tools/deflate_tokens.py [n_pairs]   # bench's configs[4] masks and images
"""
import struct
import sys
import zlib

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DEXT = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]
CLORD = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self, b):
        self.v = int.from_bytes(b, "little")
        self.p = 0

    def get(self, n):
        r = (self.v >> self.p) & ((1 << n) - 1)
        self.p += n
        return r


def table(lens):
    codes, code, bl = {}, 0, [0] * 16
    for l in lens:
        bl[l] += 1
    bl[0] = 0
    nxt, code = [0] * 16, 0
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    for s, l in enumerate(lens):
        if l:
            codes[(l, nxt[l])] = s
            nxt[l] += 1
    return codes


def sym(bits, t):
    c, l = 0, 0
    while True:
        c = (c << 1) | bits.get(1)
        l += 1
        if (l, c) in t:
            return t[(l, c)]


def tokens(z):
    bits = Bits(z[2:])
    st = dict(blocks=0, lit=0, match=0, d1=0, dge=0, dlt=0, out=0, stored=0)
    while True:
        last, typ = bits.get(1), bits.get(2)
        st["blocks"] += 1
        if typ == 0:
            bits.p = (bits.p + 7) & ~7
            n = bits.get(16)
            bits.get(16)
            bits.p += 8 * n
            st["stored"] += n
            st["out"] += n
        else:
            if typ == 1:
                tl = table([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8)
                td = table([5] * 30)
            else:
                hl, hd, hc = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
                cl = [0] * 19
                for i in range(hc):
                    cl[CLORD[i]] = bits.get(3)
                tc = table(cl)
                lens = []
                while len(lens) < hl + hd:
                    s = sym(bits, tc)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + bits.get(2))
                    elif s == 17:
                        lens += [0] * (3 + bits.get(3))
                    else:
                        lens += [0] * (11 + bits.get(7))
                tl, td = table(lens[:hl]), table(lens[hl:])
            while True:
                s = sym(bits, tl)
                if s < 256:
                    st["lit"] += 1
                    st["out"] += 1
                    continue
                if s == 256:
                    break
                ln = LBASE[s - 257] + bits.get(LEXT[s - 257])
                ds = sym(bits, td)
                dbase = 1 if ds < 4 else (1 << (ds // 2)) + 1 + ((ds & 1) << (ds // 2 - 1))
                d = dbase + bits.get(DEXT[ds])
                st["match"] += 1
                st["out"] += ln
                st["d1" if d == 1 else "dge" if d >= ln else "dlt"] += 1
        if last:
            return st


def png_idat(data):
    p, z = 8, b""
    while p < len(data):
        n, t = struct.unpack(">I4s", data[p:p + 8])
        if t == b"IDAT":
            z += data[p + 8:p + 8 + n]
        p += 12 + n
    return z


if __name__ == "__main__":
    sys.path.insert(0, ".")
    import bench
    from datago_amd import synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    spec = synth.mixed_spec(0, n, 256, 2048)
    for i in range(n):
        img, mask = bench.png_pair((i, spec[i]))
        for name, d in (("mask", mask),):
            z = png_idat(d)
            st = tokens(z)
            assert st["out"] == len(zlib.decompress(z))
            print(name, spec[i][:2], "zlen", len(z), st)
