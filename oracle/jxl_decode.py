"""ORACLE decoder (test infrastructure only -- never part of the product path).

A minimal JPEG XL codestream decoder for the subset the encoder writes:
bare codestream (0xFF0A), SizeHeader, all-default ImageMetadata (8-bit sRGB,
xyb_encoded), one VarDCT frame with 8x8-class AC strategies, default
quantization tables / block context map / coefficient orders, modular LF
groups with local MA trees, prefix-code or ANS entropy streams, no LZ77, no
loop filters.

It is written from the decoder's side of the format ([ext] ISO/IEC 18181-1 /
libjxl dec_*.cc; neither is in /root/reference, so parity with djxl is
unpinned) and is the independent read-back that pins the encoder's bitstream
layout: every test decodes the produced bytes, checks that the recovered
AC strategies / quant field / quantized coefficients equal the encoder's, and
measures PSNR with the reference harness formula
(benchmark-jpegxl/src/image_reader.rs:555-606).
"""
from __future__ import annotations

import math

import numpy as np


LAST_TOC = None  # (byte offsets, sizes) of the last decoded codestream's sections


class JxlError(Exception):
    pass


# ----------------------------------------------------------------------------
# bit reader
# ----------------------------------------------------------------------------
class BitReader:
    def __init__(self, data: bytes, start_bit: int = 0, end_bit: int | None = None):
        self.data = bytes(data) + b"\0" * 16
        self.pos = start_bit
        self.end = len(data) * 8 if end_bit is None else end_bit

    def read(self, n: int) -> int:
        if n == 0:
            return 0
        p = self.pos >> 3
        v = int.from_bytes(self.data[p:p + 9], "little") >> (self.pos & 7)
        self.pos += n
        if self.pos > self.end:
            raise JxlError("read past end of section")
        return v & ((1 << n) - 1)

    def peek(self, n: int) -> int:
        p = self.pos >> 3
        v = int.from_bytes(self.data[p:p + 9], "little") >> (self.pos & 7)
        return v & ((1 << n) - 1)

    def skip(self, n: int):
        self.pos += n
        if self.pos > self.end:
            raise JxlError("read past end of section")

    def bool(self) -> bool:
        return self.read(1) == 1

    def pad(self):
        self.pos = (self.pos + 7) & ~7

    def u32(self, *dists):
        sel = self.read(2)
        d = dists[sel]
        if d[0] == "v":
            return d[1]
        return self.read(d[1]) + d[2]

    def u64(self) -> int:
        sel = self.read(2)
        if sel == 0:
            return 0
        if sel == 1:
            return 1 + self.read(4)
        if sel == 2:
            return 17 + self.read(8)
        v = self.read(12)
        shift = 12
        while self.read(1):
            if shift == 60:
                v |= self.read(4) << 60
                break
            v |= self.read(8) << shift
            shift += 8
        return v

    def f16(self) -> float:
        bits = self.read(16)
        return float(np.frombuffer(np.uint16(bits).tobytes(), dtype=np.float16)[0])


def ceil_log2(x: int) -> int:
    n = 0
    while (1 << n) < x:
        n += 1
    return n


def unpack_signed(u: int) -> int:
    return (u >> 1) ^ -(u & 1)


# ----------------------------------------------------------------------------
# entropy decoding
# ----------------------------------------------------------------------------
class PrefixCode:
    """Brotli-style canonical prefix code read LSB-first."""

    def __init__(self, lengths):
        self.single = None
        used = [(l, s) for s, l in enumerate(lengths) if l]
        if len(used) == 0:
            self.single = 0
            return
        if len(used) == 1 and used[0][0] == 0:
            self.single = used[0][1]
            return
        maxlen = max(l for l, _ in used)
        self.maxlen = maxlen
        bl = [0] * 16
        for l, _ in used:
            bl[l] += 1
        nxt = [0] * 17
        c = 0
        for b in range(1, 16):
            c = (c + bl[b - 1]) << 1
            nxt[b] = c
        table_sym = np.zeros(1 << maxlen, dtype=np.int32)
        table_len = np.zeros(1 << maxlen, dtype=np.int32)
        filled = np.zeros(1 << maxlen, dtype=bool)
        for s, l in enumerate(lengths):
            if not l:
                continue
            code = nxt[l]
            nxt[l] += 1
            rev = int(format(code, "0%db" % l)[::-1], 2)
            idx = np.arange(rev, 1 << maxlen, 1 << l)
            if filled[idx].any():
                raise JxlError("overlapping prefix code")
            table_sym[idx] = s
            table_len[idx] = l
            filled[idx] = True
        if not filled.all():
            raise JxlError("incomplete prefix code")
        self.sym = table_sym.tolist()
        self.len = table_len.tolist()

    def read(self, br: BitReader) -> int:
        if self.single is not None:
            return self.single
        idx = br.peek(self.maxlen)
        br.skip(self.len[idx])
        return self.sym[idx]


def read_simple_prefix(br: BitReader, alphabet: int):
    max_bits = (alphabet - 1).bit_length() if alphabet > 1 else 0
    nsym = br.read(2) + 1
    syms = [br.read(max_bits) for _ in range(nsym)]
    for s in syms:
        if s >= alphabet:
            raise JxlError("simple code symbol out of range")
    if len(set(syms)) != len(syms):
        raise JxlError("duplicate simple code symbols")
    lengths = [0] * alphabet
    if nsym == 1:
        return _single(syms[0])
    if nsym == 2:
        for s in syms:
            lengths[s] = 1
    elif nsym == 3:
        lengths[syms[0]] = 1
        lengths[syms[1]] = 2
        lengths[syms[2]] = 2
    else:
        if br.read(1):  # tree_select
            lengths[syms[0]] = 1
            lengths[syms[1]] = 2
            lengths[syms[2]] = 3
            lengths[syms[3]] = 3
        else:
            for s in syms:
                lengths[s] = 2
    return PrefixCode(lengths)


def _single(sym):
    p = PrefixCode([])
    p.single = sym
    return p


K_CL_ORDER = [1, 2, 3, 4, 0, 5, 17, 6, 16, 7, 8, 9, 10, 11, 12, 13, 14, 15]
# static code for code-length code lengths (4-bit peek -> (bits, value))
K_CLCL = [(2, 0), (2, 4), (2, 3), (3, 2), (2, 0), (2, 4), (2, 3), (4, 1),
          (2, 0), (2, 4), (2, 3), (3, 2), (2, 0), (2, 4), (2, 3), (4, 5)]


def read_prefix_code(br: BitReader, alphabet: int) -> PrefixCode:
    if alphabet == 1:
        return _single(0)
    hskip = br.read(2)
    if hskip == 1:
        return read_simple_prefix(br, alphabet)
    cl = [0] * 18
    space = 32
    ncodes = 0
    i = hskip
    while i < 18 and space > 0:
        b, v = K_CLCL[br.peek(4)]
        br.skip(b)
        cl[K_CL_ORDER[i]] = v
        if v:
            space -= 32 >> v
            ncodes += 1
        i += 1
    if not (ncodes == 1 or space == 0):
        raise JxlError("invalid code-length code")
    if ncodes == 1:
        only = [s for s in range(18) if cl[s]][0]
        clcode = _single(only)
    else:
        clcode = PrefixCode(cl)
    lengths = [0] * alphabet
    sym = 0
    prev_len = 8
    repeat = 0
    repeat_len = 0
    space = 32768
    while sym < alphabet and space > 0:
        v = clcode.read(br)
        if v < 16:
            repeat = 0
            lengths[sym] = v
            sym += 1
            if v:
                prev_len = v
                space -= 32768 >> v
        else:
            extra = 2 if v == 16 else 3
            new_len = prev_len if v == 16 else 0
            if repeat_len != new_len:
                repeat = 0
                repeat_len = new_len
            old = repeat
            if repeat > 0:
                repeat = (repeat - 2) << extra
            repeat += br.read(extra) + 3
            delta = repeat - old
            if sym + delta > alphabet:
                raise JxlError("code length repeat overflow")
            for k in range(delta):
                lengths[sym + k] = repeat_len
            sym += delta
            if repeat_len:
                space -= delta << (15 - repeat_len)
    if space != 0:
        raise JxlError("incomplete prefix code lengths")
    return PrefixCode(lengths)


class UintConfig:
    def __init__(self, split_exp, msb, lsb):
        self.split_exp, self.msb, self.lsb = split_exp, msb, lsb
        self.split = 1 << split_exp

    def read(self, token: int, br: BitReader) -> int:
        if token < self.split:
            return token
        ml = self.msb + self.lsb
        nbits = self.split_exp - ml + ((token - self.split) >> ml)
        low = token & ((1 << self.lsb) - 1)
        token >>= self.lsb
        bits = br.read(nbits)
        hi = (token & ((1 << self.msb) - 1)) | (1 << self.msb)
        return (((hi << nbits) | bits) << self.lsb) | low


def read_uint_config(br: BitReader, log_alpha: int) -> UintConfig:
    split_exp = br.read(ceil_log2(log_alpha + 1))
    msb = lsb = 0
    if split_exp != log_alpha:
        msb = br.read(ceil_log2(split_exp + 1))
        if msb > split_exp:
            raise JxlError("bad uint config")
        lsb = br.read(ceil_log2(split_exp - msb + 1))
        if msb + lsb > split_exp:
            raise JxlError("bad uint config")
    return UintConfig(split_exp, msb, lsb)


def read_varlen_u8(br: BitReader) -> int:
    if br.read(1):
        n = br.read(3)
        if n == 0:
            return 1
        return br.read(n) + (1 << n)
    return 0


def read_varlen_u16(br: BitReader) -> int:
    if br.read(1):
        n = br.read(4)
        if n == 0:
            return 1
        return br.read(n) + (1 << n)
    return 0


# ANS: 12-bit precision, alias tables [ext dec_ans.cc]
ANS_LOG_TAB = 12
LOGCOUNT_CODE = {0: (5, 17), 1: (4, 11), 2: (4, 15), 3: (4, 3), 4: (4, 9), 5: (4, 7),
                 6: (3, 4), 7: (3, 2), 8: (3, 5), 9: (3, 6), 10: (3, 0), 11: (6, 33),
                 12: (7, 1), 13: (7, 65)}
_LOGCOUNT_TABLE = {}
for _sym, (_l, _c) in LOGCOUNT_CODE.items():
    for _hi in range(1 << (7 - _l)):
        _LOGCOUNT_TABLE[_c | (_hi << _l)] = (_l, _sym)


def pop_count_precision(logcount: int, shift: int) -> int:
    r = min(logcount, shift - ((ANS_LOG_TAB - logcount) >> 1))
    return max(r, 0)


def read_ans_histogram(br: BitReader):
    total = 1 << ANS_LOG_TAB
    if br.read(1):  # simple
        nsym = br.read(1) + 1
        syms = [read_varlen_u8(br) for _ in range(nsym)]
        counts = [0] * (max(syms) + 1)
        if nsym == 1:
            counts[syms[0]] = total
        else:
            if syms[0] == syms[1]:
                raise JxlError("bad simple ANS histogram")
            counts[syms[0]] = br.read(ANS_LOG_TAB)
            counts[syms[1]] = total - counts[syms[0]]
        return counts
    if br.read(1):  # flat
        alpha = read_varlen_u8(br) + 1
        base, rem = divmod(total, alpha)
        return [base + (1 if i < rem else 0) for i in range(alpha)]
    upper = (ANS_LOG_TAB + 1).bit_length() - 1
    log = 0
    while log < upper and br.read(1):
        log += 1
    shift = (br.read(log) | (1 << log)) - 1
    if shift > ANS_LOG_TAB + 1:
        raise JxlError("bad shift")
    length = read_varlen_u8(br) + 3
    logcounts = [0] * length
    same = [0] * length
    omit_log, omit_pos = -1, -1
    i = 0
    while i < length:
        nb, v = _LOGCOUNT_TABLE[br.peek(7)]
        br.skip(nb)
        logcounts[i] = v
        if v == ANS_LOG_TAB + 1:
            rle = read_varlen_u8(br)
            same[i] = rle + 5
            i += rle + 4
            continue
        if v > omit_log:
            omit_log, omit_pos = v, i
        i += 1
    if omit_pos < 0:
        raise JxlError("bad histogram")
    if omit_pos + 1 < length and logcounts[omit_pos + 1] == ANS_LOG_TAB + 1:
        raise JxlError("bad histogram")
    counts = [0] * length
    prev = 0
    numsame = 0
    tot = 0
    for i in range(length):
        if same[i]:
            numsame = same[i] - 1
            prev = counts[i - 1] if i > 0 else 0
        if numsame > 0:
            counts[i] = prev
            numsame -= 1
        else:
            code = logcounts[i]
            if i == omit_pos or code == 0:
                continue
            if code == 1:
                counts[i] = 1
            else:
                bc = pop_count_precision(code - 1, shift)
                counts[i] = (1 << (code - 1)) + (br.read(bc) << (code - 1 - bc))
        tot += counts[i]
    counts[omit_pos] = total - tot
    if counts[omit_pos] <= 0:
        raise JxlError("bad histogram sum")
    return counts


def alias_table(counts, log_alpha):
    table_size = 1 << log_alpha
    entry = (1 << ANS_LOG_TAB) >> log_alpha
    counts = list(counts) + [0] * (table_size - len(counts))
    if len(counts) > table_size:
        raise JxlError("histogram larger than alphabet")
    nz = [i for i, c in enumerate(counts) if c]
    cutoff = [0] * table_size
    right = [0] * table_size
    offset = [0] * table_size
    if len(nz) == 1:
        s = nz[0]
        for i in range(table_size):
            right[i] = s
            offset[i] = i * entry
            cutoff[i] = 0
        return cutoff, right, offset, entry
    cut = counts[:]
    under, over = [], []
    for i in range(table_size):
        if cut[i] > entry:
            over.append(i)
        elif cut[i] < entry:
            under.append(i)
    while over:
        o = over[-1]
        u = under.pop()
        by = entry - cut[u]
        cut[o] -= by
        right[u] = o
        offset[u] = cut[o]
        if cut[o] < entry:
            over.pop()
            under.append(o)
        elif cut[o] == entry:
            over.pop()
    for i in range(table_size):
        if cut[i] == entry:
            right[i] = i
            offset[i] = 0
            cutoff[i] = 0
        else:
            offset[i] -= cut[i]
            cutoff[i] = cut[i]
    return cutoff, right, offset, entry


class EntropyStream:
    """DecodeHistograms + a symbol reader (prefix or ANS)."""

    def __init__(self, br: BitReader, nctx: int):
        if br.read(1):
            raise JxlError("LZ77 streams are not produced by this encoder")
        if nctx > 1:
            self.ctxmap = read_context_map(br, nctx)
        else:
            self.ctxmap = [0]
        nh = max(self.ctxmap) + 1
        self.prefix = br.bool()
        log_alpha = 15 if self.prefix else 5 + br.read(2)
        self.cfgs = [read_uint_config(br, log_alpha) for _ in range(nh)]
        if self.prefix:
            alphas = [read_varlen_u16(br) + 1 for _ in range(nh)]
            self.codes = [read_prefix_code(br, a) for a in alphas]
        else:
            self.tables = []
            self.freqs = []
            for _ in range(nh):
                counts = read_ans_histogram(br)
                if len(counts) > (1 << log_alpha):
                    raise JxlError("ANS histogram too large")
                self.freqs.append(counts + [0] * ((1 << log_alpha) - len(counts)))
                self.tables.append(alias_table(counts, log_alpha))
            self.log_alpha = log_alpha
        self.state = None

    def begin(self, br: BitReader):
        if not self.prefix:
            self.state = br.read(32)

    def read_symbol(self, br: BitReader, h: int) -> int:
        if self.prefix:
            return self.codes[h].read(br)
        cutoff, right, offset, entry = self.tables[h]
        res = self.state & 0xFFF
        i = res // entry
        pos = res % entry
        if pos >= cutoff[i]:
            sym = right[i]
            off = offset[i] + pos
        else:
            sym = i
            off = pos
        self.state = self.freqs[h][sym] * (self.state >> 12) + off
        if self.state < (1 << 16):
            self.state = ((self.state << 16) | br.read(16)) & 0xFFFFFFFF
        return sym

    def read(self, br: BitReader, ctx: int) -> int:
        h = self.ctxmap[ctx]
        tok = self.read_symbol(br, h)
        return self.cfgs[h].read(tok, br)

    def end(self):
        if not self.prefix and self.state != 0x130000:
            raise JxlError("ANS final state mismatch: %x" % self.state)


def read_context_map(br: BitReader, n: int):
    if br.read(1):  # simple
        bits = br.read(2)
        cm = [br.read(bits) for _ in range(n)]
    else:
        use_mtf = br.read(1)
        es = EntropyStream(br, 1)
        es.begin(br)
        cm = [es.read(br, 0) for _ in range(n)]
        es.end()
        if use_mtf:
            mtf = list(range(256))
            out = []
            for v in cm:
                s = mtf[v]
                out.append(s)
                if v:
                    mtf.pop(v)
                    mtf.insert(0, s)
            cm = out
    nh = max(cm) + 1
    if len(set(cm)) != nh:
        raise JxlError("incomplete context map")
    return cm


# ----------------------------------------------------------------------------
# modular sub-bitstreams
# ----------------------------------------------------------------------------
def read_tree(br: BitReader):
    es = EntropyStream(br, 6)
    es.begin(br)
    nodes = []
    to_decode = 1
    leaf_id = 0
    while to_decode > 0:
        to_decode -= 1
        prop = es.read(br, 1)
        if prop > 256:
            raise JxlError("bad tree property")
        if prop == 0:
            pred = es.read(br, 2)
            off = unpack_signed(es.read(br, 3))
            mlog = es.read(br, 4)
            mbits = es.read(br, 5)
            if pred > 13:
                raise JxlError("bad predictor")
            nodes.append(("leaf", leaf_id, pred, off, (mbits + 1) << mlog))
            leaf_id += 1
        else:
            sv = unpack_signed(es.read(br, 0))
            p = len(nodes)
            nodes.append(("split", prop - 1, sv, p + to_decode + 1, p + to_decode + 2))
            to_decode += 2
    es.end()
    return nodes, leaf_id


def _predict(pred, img, x, y, w):
    W = img[y][x - 1] if x > 0 else (img[y - 1][x] if y > 0 else 0)
    if pred == 1:
        return W
    N = img[y - 1][x] if y > 0 else W
    if pred == 2:
        return N
    NW = img[y - 1][x - 1] if (x > 0 and y > 0) else W
    if pred == 3:
        return (W + N) // 2
    if pred == 5:
        g = W + N - NW
        lo, hi = min(W, N), max(W, N)
        return min(max(g, lo), hi)
    if pred == 8:
        return NW
    raise JxlError("predictor %d not supported by the test decoder" % pred)


def read_modular(br: BitReader, channels):
    """channels: list of (w, h).  Returns list of 2-D int lists."""
    if br.read(1):
        raise JxlError("global tree not produced by this encoder")
    if not br.read(1):
        raise JxlError("custom weighted-predictor header not produced")
    ntr = br.u32(("v", 0), ("v", 1), ("b", 4, 2), ("b", 8, 18))
    if ntr:
        raise JxlError("modular transforms not produced")
    nodes, nleaves = read_tree(br)
    es = EntropyStream(br, nleaves)
    es.begin(br)
    out = []
    for ci, (w, h) in enumerate(channels):
        img = [[0] * w for _ in range(h)]
        if w and h:
            for y in range(h):
                for x in range(w):
                    n = nodes[0]
                    i = 0
                    while n[0] == "split":
                        prop = n[1]
                        if prop == 0:
                            v = ci
                        elif prop == 2:
                            v = y
                        elif prop == 3:
                            v = x
                        else:
                            raise JxlError("property %d unsupported" % prop)
                        i = n[3] if v > n[2] else n[4]
                        n = nodes[i]
                    _, leaf, pred, off, mul = n
                    r = unpack_signed(es.read(br, leaf))
                    p = 0 if pred == 0 else _predict(pred, img, x, y, w)
                    img[y][x] = r * mul + off + p
        out.append(img)
    es.end()
    return out


# ----------------------------------------------------------------------------
# VarDCT constants (decoder view)
# ----------------------------------------------------------------------------
STRATEGY_ORDER = [0, 1, 1, 1, 2, 3, 4, 4, 5, 5, 6, 6, 1, 1, 1, 1, 1, 1, 7, 8, 8, 9, 10, 10, 11, 12, 12]
DEFAULT_CTX_MAP = [0, 1, 2, 2, 3, 3, 4, 5, 6, 6, 6, 6, 6,
                   7, 8, 9, 9, 10, 11, 12, 13, 14, 14, 14, 14, 14,
                   7, 8, 9, 9, 10, 11, 12, 13, 14, 14, 14, 14, 14]
FREQ_CTX = [0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 15, 16, 16, 17, 17, 18, 18,
            19, 19, 20, 20, 21, 21, 22, 22, 23, 23, 23, 23, 24, 24, 24, 24, 25, 25, 25, 25, 26,
            26, 26, 26, 27, 27, 27, 27, 28, 28, 28, 28, 29, 29, 29, 29, 30, 30, 30, 30]
NNZ_CTX = [0, 0, 31, 62, 62, 93, 93, 93, 93, 123, 123, 123, 123, 152, 152, 152, 152, 152,
           152, 152, 152, 180, 180, 180, 180, 180, 180, 180, 180, 180, 180, 180, 180] + [206] * 31
QUANT_BIAS = (1.0 - 0.05465007330715401, 1.0 - 0.07005449891748593,
              1.0 - 0.049935103337343655, 0.145)
M_LF = (1.0 / 4096, 1.0 / 512, 1.0 / 256)
OPSIN_BIAS = 0.0037930732552754493
OPSIN_M = np.array([[0.30, 0.622, 0.078], [0.23, 0.692, 0.078],
                    [0.24342268924547819, 0.20476744424496821, 0.55180986650955360]])


def natural_order8():
    order = [0]
    for i in range(8):
        for j in range(i + 1):
            x, y = j, i - j
            if i % 2:
                x, y = y, x
            if x == 0 and y == 0:
                continue
            order.append(y * 8 + x)
    for ip in range(7, 0, -1):
        i = ip - 1
        for j in range(i + 1):
            x, y = 7 - (i - j), 7 - j
            if i % 2:
                x, y = y, x
            order.append(y * 8 + x)
    return order


def _weights(rows, cols, bands_in, nb):
    out = np.zeros((3, rows * cols))
    for c in range(3):
        bands = [bands_in[c][0]]
        for i in range(1, nb):
            v = bands_in[c][i]
            bands.append(bands[-1] * (1 + v if v > 0 else 1 / (1 - v)))
        scale = (nb - 1) / (math.sqrt(2) + 1e-6)
        for y in range(rows):
            for x in range(cols):
                pos = math.hypot(x * scale / (cols - 1), y * scale / (rows - 1))
                idx = min(int(pos), nb - 2)
                frac = pos - idx
                a, b = bands[idx], bands[idx + 1]
                out[c, y * cols + x] = a * (b / a) ** frac
    return out


def default_dequant():
    """[kind] -> (3,64) dequant multipliers (1/weight) in coefficient layout."""
    w8 = _weights(8, 8, [[3150.0, 0.0, -0.4, -0.4, -0.4, -2.0], [560.0, 0.0, -0.3, -0.3, -0.3, -0.3],
                         [512.0, -2.0, -1.0, 0.0, -1.0, -2.0]], 6)
    w4 = _weights(4, 4, [[2200.0, 0.0, 0.0, 0.0], [392.0, 0.0, 0.0, 0.0], [112.0, -0.25, -0.25, -0.5]], 4)
    w48 = _weights(4, 8, [[2198.050556016380522, -0.96269623020744692, -0.76194253026666783, -0.6551140670773547],
                          [764.3655248643528689, -0.92630200888366945, -0.9675229603596517, -0.27845290869168118],
                          [527.107573587542228, -1.4594385811273854, -1.450082094097871593, -1.5843722511996204]], 4)
    k4 = np.zeros((3, 64))
    k48 = np.zeros((3, 64))
    for y in range(8):
        for x in range(8):
            k4[:, y * 8 + x] = w4[:, (y // 2) * 4 + x // 2]
            k48[:, y * 8 + x] = w48[:, (y // 2) * 8 + x]
    # IDENTITY / DCT2X2 [ext quant_weights.cc kQuantModeID / kQuantModeDCT2 defaults]
    idw = [[280.0, 3160.0, 3160.0], [60.0, 864.0, 864.0], [18.0, 200.0, 200.0]]
    d2w = [[3840.0, 2560.0, 1280.0, 640.0, 480.0, 300.0], [960.0, 640.0, 320.0, 180.0, 140.0, 120.0],
           [640.0, 320.0, 128.0, 64.0, 32.0, 16.0]]
    kid = np.zeros((3, 64))
    kd2 = np.zeros((3, 64))
    for c in range(3):
        kid[c, :] = idw[c][0]
        kid[c, 1] = kid[c, 8] = idw[c][1]
        kid[c, 9] = idw[c][2]
        for y in range(8):
            for x in range(8):
                if y < 2 and x < 2:
                    k = 1 if (y and x) else 0
                elif y < 4 and x < 4:
                    k = 3 if (y >= 2 and x >= 2) else 2
                else:
                    k = 5 if (y >= 4 and x >= 4) else 4
                kd2[c, y * 8 + x] = d2w[c][k]
    return {0: 1.0 / w8, 1: 1.0 / kid, 2: 1.0 / kd2, 3: 1.0 / k4, 12: 1.0 / k48, 13: 1.0 / k48}


def _idct_mat(n):
    m = np.zeros((n, n))
    for k in range(n):
        for x in range(n):
            m[x, k] = (1.0 if k == 0 else math.sqrt(2)) * math.cos(math.pi * (2 * x + 1) * k / (2 * n))
    return m  # pixels = m @ coeffs


_I8, _I4 = _idct_mat(8), _idct_mat(4)

# merged varblocks [ext AcStrategy]: raw id -> (blocks down, blocks across, kind)
SHAPES = {6: (2, 1, 0), 7: (1, 2, 0), 4: (2, 2, 1), 10: (4, 2, 2), 11: (2, 4, 2), 5: (4, 4, 3),
          19: (8, 4, 4), 20: (4, 8, 4), 18: (8, 8, 5),
          22: (16, 8, 6), 23: (8, 16, 6), 21: (16, 16, 7), 25: (32, 16, 8), 26: (16, 32, 8),
          24: (32, 32, 9)}
# default weight bands per kind [ext quant_weights.cc]; stored dims rows x cols
KIND_DIM = [(8, 16), (16, 16), (16, 32), (32, 32), (32, 64), (64, 64), (64, 128), (128, 128),
            (128, 256), (256, 256)]
KIND_BANDS = [
    [[7240.7734393502, -0.7, -0.7, -0.2, -0.2, -0.2, -0.5],
     [1448.15468787004, -0.5, -0.5, -0.5, -0.2, -0.2, -0.2],
     [506.854140754517, -1.4, -0.2, -0.5, -0.5, -1.5, -3.6]],
    [[8996.8725711814115328, -1.3000777393353804, -0.49424529824571225, -0.439093774457103443,
      -0.6350101832695744, -0.90177264050827612, -1.6162099239887414],
     [3191.48366296844234752, -0.67424582104194355, -0.80745813428471001, -0.44925837484843441,
      -0.35865440981033403, -0.31322389111877305, -0.37615025315725483],
     [1157.50408145487200256, -2.0531423165804414, -1.4, -0.50687130033378396,
      -0.42708730624733904, -1.4856834539296244, -4.9209142884401604]],
    [[13844.97076442300573, -0.97113799999999995, -0.658, -0.42026, -0.22712, -0.2206, -0.226, -0.6],
     [4798.964084220744293, -0.61125308982767057, -0.83770786552491361, -0.79014862079498627,
      -0.2692727459704829, -0.38272769465388551, -0.22924222653091453, -0.20719098826199578],
     [1807.236946760964614, -1.2, -1.2, -0.7, -0.7, -0.7, -0.4, -0.5]],
    [[15718.40830982518931456, -1.025, -0.98, -0.9012, -0.4, -0.48819395464, -0.421064, -0.27],
     [7305.7636810695983104, -0.8041958212306401, -0.7633036457487539, -0.55660379990111464,
      -0.49785304658857626, -0.43699592683512467, -0.40180866526242109, -0.27321683125358037],
     [3803.53173721215041536, -3.060733579805728, -2.0413270132490346, -2.0235650159727417,
      -0.5495389509954993, -0.4, -0.4, -0.3]],
    [[0.65 * 23629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671],
     [0.65 * 8611.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037],
     [0.65 * 4492.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5]],
    [[0.9 * 26629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671],
     [0.9 * 9311.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037],
     [0.9 * 4992.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5]],
    # DCT128X64, DCT128X128, DCT256X128, DCT256X256 (the encoder's restated
    # defaults, oracle/merge.c; parity with libjxl unpinned)
    [[1.3 * 23629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671],
     [1.3 * 8611.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037],
     [1.3 * 4492.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5]],
    [[1.7 * 26629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671],
     [1.7 * 9311.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037],
     [1.7 * 4992.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5]],
    [[2.2 * 23629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671],
     [2.2 * 8611.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037],
     [2.2 * 4492.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5]],
    [[3.0 * 26629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671],
     [3.0 * 9311.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037],
     [3.0 * 4992.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5]],
]


def natural_order(rows, cols):
    """[position] -> stored raster index of a rows x cols (rows <= cols)
    coefficient block: LLF raster first, then the y-scaled zigzag."""
    cs, cl, xf = rows // 8, cols // 8, cols // rows
    order = [y * cols + x for y in range(cs) for x in range(cl)]
    for i in range(cols):
        for j in range(i + 1):
            x, y = j, i - j
            if i % 2:
                x, y = y, x
            if y % xf:
                continue
            y //= xf
            if x < cl and y < cs:
                continue
            order.append(y * cols + x)
    for ip in range(cols - 1, 0, -1):
        i = ip - 1
        for j in range(i + 1):
            x, y = cols - 1 - (i - j), cols - 1 - j
            if i % 2:
                x, y = y, x
            if y % xf:
                continue
            y //= xf
            order.append(y * cols + x)
    assert len(order) == rows * cols and len(set(order)) == rows * cols
    return order


_KIND_CACHE = {}

# DequantMatrices [ext quant_weights.cc]: quant table index (the format's
# order DCT, IDENTITY, DCT2X2, DCT4X4, DCT16X16, DCT32X32, DCT16X8, DCT32X8,
# DCT32X16, DCT64X64, DCT64X32, DCT4X8, AFV0, DCT128X128, DCT128X64,
# DCT256X256, DCT256X128) -> merged-varblock kind (None: an 8x8-class table)
QUANT_TABLE_KIND = [None, None, None, None, 1, 3, 0, None, 2, 5, 4, None, None, 7, 6, 9, 8]
QM_LIBRARY, QM_DCT = 0, 6


def f16_value(bits):
    """binary16 bits -> float [ext F16Coder::Read]; inf / NaN are invalid"""
    sign, exp, mant = bits >> 15, (bits >> 10) & 31, bits & 1023
    if exp == 31:
        raise JxlError("binary16 inf / NaN in a header")
    v = mant * 2.0 ** -24 if exp == 0 else (1024 + mant) * 2.0 ** (exp - 25)
    return -v if sign else v


def read_dequant_matrices(br):
    """-> {kind: bands (3 x nb)} of the tables a stream writes in DCT mode;
    kinds absent from the dict use the decoder's defaults (KIND_BANDS)."""
    if br.bool():  # all_default
        return {}
    params = {}
    for t, kind in enumerate(QUANT_TABLE_KIND):
        mode = br.read(3)
        if mode == QM_LIBRARY:
            br.read(0)  # one predefined table set: zero bits
            continue
        if mode != QM_DCT or kind is None:
            raise JxlError("quant table %d: mode %d not produced" % (t, mode))
        nb = br.read(4) + 1
        bands = []
        for c in range(3):
            row = [f16_value(br.read(16)) for _ in range(nb)]
            if row[0] < 1e-8:
                raise JxlError("quant table %d: first band ~0" % t)
            row[0] *= 64.0
            bands.append(row)
        params[kind] = bands
    return params


def kind_tables(kind, bands=None):
    """(inverse weights (3, rows*cols) stored raster, natural order); bands:
    the stream's parameters for the kind (read_dequant_matrices), else the
    library defaults"""
    key = (kind, None if bands is None else tuple(tuple(r) for r in bands))
    if key not in _KIND_CACHE:
        r, c = KIND_DIM[kind]
        src = KIND_BANDS[kind] if bands is None else bands
        w = _weights(r, c, src, len(src[0]))
        _KIND_CACHE[key] = (1.0 / w, natural_order(r, c))
    return _KIND_CACHE[key]


def _llf_scale(M):
    return np.array([math.cos(math.pi * k / (16 * M)) * math.cos(math.pi * k / (8 * M)) *
                     math.cos(math.pi * k / (4 * M)) for k in range(M)])


def _dct_mat(n):
    """normalized forward DCT: out = m @ x, out[0] = mean"""
    return np.linalg.inv(_idct_mat(n))


def reconstruct_varblock(t, coefs, dcs):
    """coefs: (R, C) dequantized coefficients in pixel orientation (LLF slots
    ignored); dcs: (cy, cx) dequantized DC of the covered blocks -> pixels"""
    cy, cx, _ = SHAPES[t]
    co = coefs.copy()
    llf = _dct_mat(cy) @ dcs @ _dct_mat(cx).T
    llf = llf / np.outer(_llf_scale(cy), _llf_scale(cx))
    co[:cy, :cx] = llf
    return _idct_mat(8 * cy) @ co @ _idct_mat(8 * cx).T


def inverse_transform(t, co):
    """co: 64 coefficients (layout of strategy t) -> 8x8 pixels."""
    c = co.reshape(8, 8)
    if t == 0:
        return _I8 @ c @ _I8.T
    out = np.zeros((8, 8))
    if t == 2:  # DCT2X2: inverse 2x2 Haar steps, S = 2, 4, 8 [ext IDCT2TopBlock]
        cur = c.copy()
        for S in (2, 4, 8):
            n = S // 2
            nxt = cur.copy()
            for y in range(n):
                for x in range(n):
                    c00, c01 = cur[y, x], cur[y, n + x]
                    c10, c11 = cur[n + y, x], cur[n + y, n + x]
                    nxt[2 * y, 2 * x] = c00 + c01 + c10 + c11
                    nxt[2 * y, 2 * x + 1] = c00 + c01 - c10 - c11
                    nxt[2 * y + 1, 2 * x] = c00 - c01 + c10 - c11
                    nxt[2 * y + 1, 2 * x + 1] = c00 - c01 - c10 + c11
            cur = nxt
        return cur
    if t == 1:  # IDENTITY [ext dec_transforms IDENTITY]
        A, B, C, D = c[0, 0], c[0, 1], c[1, 0], c[1, 1]
        dcs = [A + B + C + D, A + B - C - D, A - B + C - D, A - B - C + D]
        for sy in range(2):
            for sx in range(2):
                res = np.array([[c[sy + 2 * iy, sx + 2 * ix] for ix in range(4)] for iy in range(4)])
                p11 = dcs[sy * 2 + sx] - (res.sum() - res[0, 0]) / 16.0
                blk = res + p11
                blk[1, 1] = p11
                blk[0, 0] = res[1, 1] + p11
                out[4 * sy:4 * sy + 4, 4 * sx:4 * sx + 4] = blk
        return out
    if t == 3:
        A, B, C, D = c[0, 0], c[0, 1], c[1, 0], c[1, 1]
        dcs = [A + B + C + D, A + B - C - D, A - B + C - D, A - B - C + D]
        for sy in range(2):
            for sx in range(2):
                blk = np.zeros((4, 4))
                for iy in range(4):
                    for ix in range(4):
                        blk[iy, ix] = c[sy + 2 * iy, sx + 2 * ix]
                blk[0, 0] = dcs[sy * 2 + sx]
                out[4 * sy:4 * sy + 4, 4 * sx:4 * sx + 4] = _I4 @ blk @ _I4.T
        return out
    d0, d1 = c[0, 0], c[1, 0]
    dcs = [d0 + d1, d0 - d1]
    if t == 13:  # DCT8X4: two 4x8 (rows x cols) halves stacked
        for sy in range(2):
            blk = np.zeros((4, 8))
            for iy in range(4):
                blk[iy, :] = c[sy + 2 * iy, :]
            blk[0, 0] = dcs[sy]
            out[4 * sy:4 * sy + 4, :] = _I4 @ blk @ _I8.T
        return out
    if t == 12:  # DCT4X8: two 8x4 halves side by side, coefficients transposed
        for sx in range(2):
            blk = np.zeros((8, 4))  # [row freq][col freq]
            for cx in range(4):
                blk[:, cx] = c[sx + 2 * cx, :]
            blk[0, 0] = dcs[sx]
            out[:, 4 * sx:4 * sx + 4] = _I8 @ blk @ _I4.T
        return out
    raise JxlError("AC strategy %d not supported by the test decoder" % t)


def xyb_to_srgb8(X, Y, B):
    cb = OPSIN_BIAS ** (1.0 / 3.0)
    L = Y + X + cb
    M = Y - X + cb
    S = B + cb
    mixed = np.stack([L ** 3 - OPSIN_BIAS, M ** 3 - OPSIN_BIAS, S ** 3 - OPSIN_BIAS], axis=-1)
    lin = mixed @ np.linalg.inv(OPSIN_M).T
    lin = np.clip(lin, 0.0, 1.0)
    srgb = np.where(lin <= 0.0031308, lin * 12.92, 1.055 * np.power(lin, 1 / 2.4) - 0.055)
    return np.clip(np.floor(srgb * 255.0 + 0.5), 0, 255).astype(np.uint8)


# ----------------------------------------------------------------------------
# frame decoding
# ----------------------------------------------------------------------------
def _read_size(br):
    return br.u32(("b", 9, 1), ("b", 13, 1), ("b", 18, 1), ("b", 30, 1))


class Decoded:
    pass


def decode(data: bytes, want_pixels: bool = True, groups=None, toc_only: bool = False) -> Decoded:
    """groups: decode only these pass groups (and the LF groups holding them;
    every other block stays zero, no pixels) -- for spot checks of large
    frames, whose full decode takes minutes in Python."""
    br = BitReader(data)
    if br.read(16) != 0x0AFF:
        raise JxlError("not a JPEG XL codestream")
    if br.bool():
        ys = (br.read(5) + 1) * 8
        ratio = br.read(3)
        if ratio:
            raise JxlError("ratio sizes not produced")
        xs = (br.read(5) + 1) * 8
    else:
        ys = _read_size(br)
        if br.read(3):
            raise JxlError("ratio sizes not produced")
        xs = _read_size(br)
    if not br.bool():
        raise JxlError("only all-default ImageMetadata is produced")
    br.pad()
    # FrameHeader
    if br.bool():
        raise JxlError("all-default frame header not produced")
    ftype = br.read(2)
    enc = br.read(1)
    flags = br.u64()
    if ftype != 0 or enc != 0:
        raise JxlError("only regular VarDCT frames")
    if flags != 128:
        raise JxlError("unexpected frame flags %d" % flags)
    if br.u32(("v", 1), ("v", 2), ("v", 4), ("v", 8)) != 1:
        raise JxlError("upsampling")
    x_qm = br.read(3)
    b_qm = br.read(3)
    if br.u32(("v", 1), ("v", 2), ("v", 3), ("b", 3, 4)) != 1:
        raise JxlError("passes")
    if br.bool():
        raise JxlError("crop")
    if br.u32(("v", 0), ("v", 1), ("v", 2), ("b", 2, 3)) != 0:
        raise JxlError("blending")
    if not br.bool():
        raise JxlError("is_last")
    nlen = br.u32(("v", 0), ("b", 4, 0), ("b", 5, 16), ("b", 10, 48))
    br.skip(8 * nlen)
    # LoopFilter [ext loop_filter.h]: all_default = Gaborish + one EPF iteration
    if br.bool():
        gab, epf = True, 1
    else:
        gab = br.bool()
        if gab and br.bool():
            raise JxlError("custom Gaborish weights not produced")
        epf = br.read(2)
        if epf:
            if br.bool():
                raise JxlError("custom EPF sharpness LUT not produced")
            if br.bool():
                raise JxlError("custom EPF channel scales not produced")
            if br.bool():
                raise JxlError("custom EPF sigmas not produced")
        if br.u64():
            raise JxlError("loop filter extensions")
    if br.u64():
        raise JxlError("frame extensions")
    bxs, bys = (xs + 7) // 8, (ys + 7) // 8
    gxs, gys = (xs + 255) // 256, (ys + 255) // 256
    ng = gxs * gys
    lfxs, lfys = (xs + 2047) // 2048, (ys + 2047) // 2048
    nlf = lfxs * lfys
    # TOC
    if br.bool():
        raise JxlError("permuted TOC not produced")
    br.pad()
    nent = 1 if ng == 1 else 2 + nlf + ng
    sizes = [br.u32(("b", 10, 0), ("b", 14, 1024), ("b", 22, 17408), ("b", 30, 4211712)) for _ in range(nent)]
    br.pad()
    base = br.pos >> 3
    if base + sum(sizes) > len(data):
        raise JxlError("truncated codestream: need %d bytes, have %d" % (base + sum(sizes), len(data)))
    offs = []
    o = base
    for s in sizes:
        offs.append(o)
        o += s
    global LAST_TOC
    LAST_TOC = (list(offs), list(sizes))  # (diagnostics: tools/diag_sections.py)

    def sec(i):
        if nent == 1:
            return shared
        return BitReader(data, offs[i] * 8, (offs[i] + sizes[i]) * 8)

    shared = BitReader(data, base * 8, (base + sizes[0]) * 8) if nent == 1 else None
    d = Decoded()
    d.xsize, d.ysize, d.bxs, d.bys = xs, ys, bxs, bys
    d.gab, d.epf_iters = bool(gab), int(epf)
    d.sharpness = np.zeros((bys, bxs), dtype=np.int32)
    d.section_sizes = sizes
    d.section_offsets = offs
    if toc_only:  # headers and TOC only (section comparisons of large frames)
        return d
    # LfGlobal
    s = sec(0)
    if not s.bool():
        raise JxlError("custom LF dequant not produced")
    G = s.u32(("b", 11, 1), ("b", 11, 2049), ("b", 12, 4097), ("b", 16, 8193))
    qdc = s.u32(("v", 16), ("b", 5, 1), ("b", 8, 1), ("b", 16, 1))
    if not s.bool():
        raise JxlError("custom block ctx map not produced")
    if not s.bool():
        raise JxlError("custom colour correlation not produced")
    if s.bool():
        raise JxlError("global tree not produced")
    d.global_scale, d.quant_dc = G, qdc
    d.dc = np.zeros((3, bys, bxs), dtype=np.int64)
    d.acs = np.zeros((bys, bxs), dtype=np.int32)
    d.qf = np.zeros((bys, bxs), dtype=np.int32)
    # chroma from luma: int8 (ytox, ytob) per 64x64 colour tile
    d.cmap = np.zeros((2, (bys + 7) // 8, (bxs + 7) // 8), dtype=np.int32)
    gsel = None if groups is None else set(int(g) for g in groups)
    if gsel is not None:
        want_pixels = False
        lfsel = set(((g // gxs) // 8) * lfxs + (g % gxs) // 8 for g in gsel)
    for lg in range(nlf):
        if gsel is not None and lg not in lfsel:
            continue
        s = sec(1 + lg)
        lgx, lgy = lg % lfxs, lg // lfxs
        bx0, by0 = lgx * 256, lgy * 256
        bw, bh = min(256, bxs - bx0), min(256, bys - by0)
        if s.read(2):
            raise JxlError("extra_precision not produced")
        ch = read_modular(s, [(bw, bh)] * 3)
        for mi, c in enumerate((1, 0, 2)):
            d.dc[c, by0:by0 + bh, bx0:bx0 + bw] = np.array(ch[mi], dtype=np.int64)
        count = s.read(ceil_log2(bw * bh)) + 1
        cw, chh = (bw + 7) // 8, (bh + 7) // 8
        meta = read_modular(s, [(cw, chh), (cw, chh), (count, 2), (bw, bh)])
        for i in range(2):
            m = np.array(meta[i], dtype=np.int32)
            if m.min() < -128 or m.max() > 127:
                raise JxlError("CfL factor out of int8 range")
            d.cmap[i, by0 // 8:by0 // 8 + chh, bx0 // 8:bx0 // 8 + cw] = m
        sh = np.array(meta[3], dtype=np.int32).reshape(bh, bw)
        if sh.min() < 0 or sh.max() > 7:
            raise JxlError("EPF sharpness out of range")
        d.sharpness[by0:by0 + bh, bx0:bx0 + bw] = sh
        k = 0
        covered = np.zeros((bh, bw), dtype=bool)
        for y in range(bh):
            for x in range(bw):
                if covered[y, x]:
                    continue
                if k >= count:
                    raise JxlError("too few varblocks")
                t = meta[2][0][k]
                if t not in (0, 1, 2, 3, 12, 13) and t not in SHAPES:
                    raise JxlError("AC strategy %d not produced" % t)
                cy, cx = SHAPES[t][:2] if t in SHAPES else (1, 1)
                if y + cy > bh or x + cx > bw or covered[y:y + cy, x:x + cx].any():
                    raise JxlError("varblock out of bounds / overlapping")
                qv = 1 + min(max(meta[2][1][k], 0), 255)
                for iy in range(cy):
                    for ix in range(cx):
                        d.acs[by0 + y + iy, bx0 + x + ix] = t | (0x80 if (iy or ix) else 0)
                        d.qf[by0 + y + iy, bx0 + x + ix] = qv
                covered[y:y + cy, x:x + cx] = True
                k += 1
        if k != count:
            raise JxlError("varblock count mismatch")
    # HfGlobal
    s = sec(1 + nlf)
    d.qm_params = read_dequant_matrices(s)
    npresets = s.read(ceil_log2(ng)) + 1
    used_orders = s.u32(("v", 0x5F), ("v", 0x13), ("v", 0), ("b", 13, 0))
    if used_orders:
        raise JxlError("custom coefficient orders not produced")
    nctx_ac = 15 * (37 + 458)
    hf = EntropyStream(s, npresets * nctx_ac)
    d.npresets = npresets
    d.group_presets = np.zeros(ng, dtype=np.int64)
    d.ac = np.zeros((bys, bxs, 3, 64), dtype=np.int64)
    d.ac_tokens = np.zeros((ng, 3), dtype=np.int64)
    for g in range(ng):
        if gsel is not None and g not in gsel:
            continue
        s = sec(2 + nlf + g)
        gx, gy = g % gxs, g // gxs
        bx0, by0 = gx * 32, gy * 32
        gw, gh = min(32, bxs - bx0), min(32, bys - by0)
        preset = s.read(ceil_log2(npresets))
        if preset >= npresets:
            raise JxlError("HF preset index out of range")
        d.group_presets[g] = preset
        off = preset * nctx_ac
        hf.begin(s)
        nzs = np.zeros((3, gh, gw), dtype=np.int64)
        for by in range(gh):
            for bx in range(gw):
                t = int(d.acs[by0 + by, bx0 + bx])
                if t & 0x80:
                    continue
                cy, cx = SHAPES[t][:2] if t in SHAPES else (1, 1)
                cb = cy * cx
                lcb = cb.bit_length() - 1
                size = 64 * cb
                ordi = STRATEGY_ORDER[t]
                for c in (1, 0, 2):
                    if bx == 0:
                        pred = 32 if by == 0 else nzs[c, by - 1, bx]
                    elif by == 0:
                        pred = nzs[c, by, bx - 1]
                    else:
                        pred = (nzs[c, by - 1, bx] + nzs[c, by, bx - 1] + 1) // 2
                    bctx = DEFAULT_CTX_MAP[(c ^ 1 if c < 2 else 2) * 13 + ordi]
                    pp = min(int(pred), 64)
                    bucket = pp if pp < 8 else 4 + pp // 2
                    nz = hf.read(s, off + bucket * 15 + bctx)
                    ntok = 1
                    if nz > size - cb:
                        raise JxlError("nzeros too large")
                    nzs[c, by:by + cy, bx:bx + cx] = (nz + cb - 1) >> lcb
                    zoff = off + 15 * 37 + 458 * bctx
                    prev = 0 if nz > size // 16 else 1
                    k = cb
                    left = nz
                    while k < size and left > 0:
                        u = hf.read(s, zoff + (NNZ_CTX[(left + cb - 1) >> lcb] + FREQ_CTX[k >> lcb]) * 2 + prev)
                        ntok += 1
                        v = unpack_signed(u)
                        sl = k >> 6
                        d.ac[by0 + by + sl // cx, bx0 + bx + sl % cx, c, k & 63] = v
                        prev = 1 if u else 0
                        left -= prev
                        k += 1
                    if left:
                        raise JxlError("nzeros not exhausted")
                    d.ac_tokens[g, c] += ntok
        hf.end()
    d.x_qm, d.b_qm = x_qm, b_qm
    if want_pixels:
        d.rgb = reconstruct(d)
    return d


def reconstruct(d: Decoded) -> np.ndarray:
    deq = default_dequant()
    qm = getattr(d, "qm_params", {})
    inv_gs = 65536.0 / d.global_scale
    x_mul = 1.25 ** (2 - d.x_qm)  # scale 2 -> 1.0
    b_mul = 1.25 ** (2 - d.b_qm)
    dc_step = [M_LF[c] * inv_gs / d.quant_dc for c in range(3)]
    X = np.zeros((d.bys * 8, d.bxs * 8))
    Y = np.zeros_like(X)
    B = np.zeros_like(X)
    ac = d.ac.astype(np.float64)
    # AdjustQuantBias
    adj = np.where(np.abs(ac) == 1, np.sign(ac) * np.array(QUANT_BIAS[:3])[None, None, :, None],
                   np.where(ac == 0, 0.0, ac - QUANT_BIAS[3] / np.where(ac == 0, 1, ac)))
    order8 = np.array(natural_order8())
    dcq = np.stack([d.dc[0] * dc_step[0], d.dc[1] * dc_step[1],
                    d.dc[2] * dc_step[2] + d.dc[1] * dc_step[1]])  # X, Y, B (ytob 1.0)
    chm = (x_mul, 1.0, b_mul)
    cmap = getattr(d, "cmap", np.zeros((2, (d.bys + 7) // 8, (d.bxs + 7) // 8), dtype=np.int32))
    for by in range(d.bys):
        for bx in range(d.bxs):
            t = int(d.acs[by, bx])
            if t & 0x80:
                continue
            qf = d.qf[by, bx]
            # colour correlation of the block's tile [ext ColorCorrelationMap:
            # base_correlation_x 0, base_correlation_b 1, colour_factor 84]
            cfx = float(np.float32(cmap[0, by // 8, bx // 8]) * np.float32(1.0 / 84.0))
            cfb = 1.0 + float(np.float32(cmap[1, by // 8, bx // 8]) * np.float32(1.0 / 84.0))
            if t in SHAPES:
                ccy, ccx, kind = SHAPES[t]
                R, C = 8 * ccy, 8 * ccx
                iw, nat = kind_tables(kind, qm.get(kind))
                nat = np.array(nat)
                cols_s = KIND_DIM[kind][1]
                sy, sx = nat // cols_s, nat % cols_s
                ky, kx = (sy, sx) if ccx >= ccy else (sx, sy)
                vals = np.zeros((3, R * C))
                for i in range(ccy * ccx):
                    vals[:, i * 64:(i + 1) * 64] = adj[by + i // ccx, bx + i % ccx]
                co = np.zeros((3, R, C))
                for c in range(3):
                    co[c, ky, kx] = vals[c] * iw[c][nat] * (inv_gs / qf) * chm[c]
                co[0] += cfx * co[1]
                co[2] += cfb * co[1]
                for c, arr in ((0, X), (1, Y), (2, B)):
                    arr[by * 8:by * 8 + R, bx * 8:bx * 8 + C] = reconstruct_varblock(
                        t, co[c], dcq[c, by:by + ccy, bx:bx + ccx])
                continue
            mul = deq[t] * (inv_gs / qf)
            raster = np.zeros((3, 64))
            raster[:, order8] = adj[by, bx]
            cy = raster[1] * mul[1]
            cx = raster[0] * mul[0] * x_mul + cfx * cy
            cb = raster[2] * mul[2] * b_mul + cfb * cy
            for arr, co, dcv in ((X, cx, dcq[0, by, bx]), (Y, cy, dcq[1, by, bx]),
                                 (B, cb, dcq[2, by, bx])):
                co = co.copy()
                co[0] = dcv
                arr[by * 8:by * 8 + 8, bx * 8:bx * 8 + 8] = inverse_transform(t, co)
    if getattr(d, "gab", False):
        X, Y, B = gaborish(X), gaborish(Y), gaborish(B)
    if getattr(d, "epf_iters", 0):
        X, Y, B = epf(X, Y, B, d)
    rgb = xyb_to_srgb8(X, Y, B)
    return rgb[:d.ysize, :d.xsize]


# ----------------------------------------------------------------------------
# restoration filters [ext: libjxl's decoder, restated from the format's
# description; constants are the LoopFilter defaults; parity with libjxl/djxl
# unpinned].  Both run on the block-padded XYB planes, mirrored at their edges
# (the encoder's inverse Gaborish, oracle/xyb.c jxo_gab_inverse, replicates the
# same edges).
# ----------------------------------------------------------------------------
GAB_W1, GAB_W2 = 0.115169525, 0.061248592
EPF_CHANNEL_SCALE = (40.0, 5.0, 3.5)
EPF_QUANT_MUL = 0.46
EPF_SHARP_LUT = tuple(i / 7.0 for i in range(8))
EPF_PASS0_SIGMA_SCALE = 0.9
EPF_PASS2_SIGMA_SCALE = 6.5
EPF_BORDER_SAD_MUL = 2.0 / 3.0
EPF_INV_SIGMA_NUM = -1.1715728752538099
EPF_MIN_SIGMA = -3.90625  # inverse sigma below this: the block is not filtered


def gaborish(P: np.ndarray) -> np.ndarray:
    """3x3 symmetric smoothing (1 centre, w1 edges, w2 corners), normalised."""
    Q = np.pad(P, 1, mode="symmetric")
    s1 = (Q[:-2, 1:-1] + Q[2:, 1:-1]) + (Q[1:-1, :-2] + Q[1:-1, 2:])
    s2 = (Q[:-2, :-2] + Q[:-2, 2:]) + (Q[2:, :-2] + Q[2:, 2:])
    return (P + GAB_W1 * s1 + GAB_W2 * s2) / (1.0 + 4.0 * GAB_W1 + 4.0 * GAB_W2)


def epf_inv_sigma(d) -> np.ndarray:
    """Per-block inverse sigma (negative; -inf-like when not filtered):
    sigma = quant_mul * sharp_lut[s] / (scale * qf * kInvSigmaNum)."""
    scale = d.global_scale / 65536.0
    lut = np.array(EPF_SHARP_LUT)[d.sharpness]
    sigma = EPF_QUANT_MUL / (scale * d.qf.astype(np.float64) * EPF_INV_SIGMA_NUM) * lut
    sigma = np.minimum(-1e-4, sigma)
    return 1.0 / sigma


def _epf_step(planes, inv_px, neigh, plus_sad, pad=3):
    Q = [np.pad(p, pad, mode="symmetric") for p in planes]
    H, W = planes[0].shape

    def sh(q, dy, dx):
        return q[pad + dy:pad + dy + H, pad + dx:pad + dx + W]

    sad_pat = ((0, 0), (-1, 0), (1, 0), (0, -1), (0, 1)) if plus_sad else ((0, 0),)
    wsum = np.ones((H, W))
    acc = [p.copy() for p in planes]
    for dy, dx in neigh:
        sad = np.zeros((H, W))
        for c in range(3):
            a = np.zeros((H, W))
            for oy, ox in sad_pat:
                a += np.abs(sh(Q[c], dy + oy, dx + ox) - sh(Q[c], oy, ox))
            sad += EPF_CHANNEL_SCALE[c] * a
        w = np.maximum(0.0, 1.0 + sad * inv_px)
        wsum += w
        for c in range(3):
            acc[c] += w * sh(Q[c], dy, dx)
    return [a / wsum for a in acc]


def epf(X, Y, B, d):
    """Edge-preserving filter, d.epf_iters passes (3: pass 0 over 12
    neighbours; >= 1: pass 1 over 4; 2-3: pass 2 with one-pixel SADs); blocks
    whose inverse sigma is below EPF_MIN_SIGMA keep their input."""
    inv_b = epf_inv_sigma(d)
    H, W = X.shape
    inv = np.repeat(np.repeat(inv_b, 8, axis=0), 8, axis=1)[:H, :W]
    skip = inv < EPF_MIN_SIGMA
    yy, xx = np.arange(H) % 8, np.arange(W) % 8
    border = ((yy == 0) | (yy == 7))[:, None] | ((xx == 0) | (xx == 7))[None, :]
    sad_mul = np.where(border, EPF_BORDER_SAD_MUL, 1.0)
    plus = ((-1, 0), (0, -1), (0, 1), (1, 0))
    steps = []
    if d.epf_iters >= 3:
        steps.append((EPF_PASS0_SIGMA_SCALE, plus + ((-1, -1), (-1, 1), (1, -1), (1, 1),
                                                     (-2, 0), (0, -2), (0, 2), (2, 0)), True))
    steps.append((1.0, plus, True))
    if d.epf_iters >= 2:
        steps.append((EPF_PASS2_SIGMA_SCALE, plus, False))
    planes = [X, Y, B]
    for scale, neigh, plus_sad in steps:
        out = _epf_step(planes, inv * sad_mul * scale, neigh, plus_sad)
        planes = [np.where(skip, p, o) for p, o in zip(planes, out)]
    return planes


def mse_psnr(orig: np.ndarray, comp: np.ndarray):
    """benchmark-jpegxl/src/image_reader.rs:555-606: f64 sum of squared sample
    differences over W*H*3 / count; PSNR = 10*log10(255^2/MSE)."""
    o = orig.astype(np.float64).ravel()
    c = comp.astype(np.float64).ravel()
    mse = float(np.sum((o - c) ** 2) / o.size)
    psnr = float("inf") if mse == 0 else 10.0 * math.log10(255.0 * 255.0 / mse)
    return mse, psnr
