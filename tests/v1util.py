"""Small pure-Python update-v1 helpers for tests (structure walking only)."""


def rd_vu(b, p):
    n = s = 0
    while True:
        x = b[p]
        p += 1
        n |= (x & 127) << s
        s += 7
        if x < 128:
            return n, p


def vu(n):
    o = bytearray()
    while n > 127:
        o.append(0x80 | (n & 127))
        n >>= 7
    o.append(n)
    return bytes(o)


def ds_offset(update: bytes) -> int:
    """Byte offset of the delete set in a *merge/diff output* (struct section re-walked via the oracle's rules)."""
    import oracle  # noqa: F401  (struct walking: lengths only)
    b = update
    p = 0
    nb, p = rd_vu(b, p)
    for _ in range(nb):
        ns, p = rd_vu(b, p)
        _, p = rd_vu(b, p)
        _, p = rd_vu(b, p)
        for _ in range(ns):
            p = _skip_struct(b, p)
    return p


def _skip_str(b, p):
    n, p = rd_vu(b, p)
    return p + n


def _skip_any(b, p):
    t = b[p]
    p += 1
    if t in (127, 126, 121, 120):
        return p
    if t == 125:
        while b[p] & 128:
            p += 1
        return p + 1
    if t == 124:
        return p + 4
    if t in (123, 122):
        return p + 8
    if t in (119, 116):
        return _skip_str(b, p)
    if t == 117:
        n, p = rd_vu(b, p)
        for _ in range(n):
            p = _skip_any(b, p)
        return p
    if t == 118:
        n, p = rd_vu(b, p)
        for _ in range(n):
            p = _skip_str(b, p)
            p = _skip_any(b, p)
        return p
    raise ValueError(t)


def _skip_struct(b, p):
    info = b[p]
    p += 1
    if info == 10 or (info & 31) == 0:
        _, p = rd_vu(b, p)
        return p
    if info & 0x80:
        _, p = rd_vu(b, p)
        _, p = rd_vu(b, p)
    if info & 0x40:
        _, p = rd_vu(b, p)
        _, p = rd_vu(b, p)
    if (info & 0xC0) == 0:
        pi, p = rd_vu(b, p)
        if pi == 1:
            p = _skip_str(b, p)
        else:
            _, p = rd_vu(b, p)
            _, p = rd_vu(b, p)
        if info & 0x20:
            p = _skip_str(b, p)
    ref = info & 31
    if ref == 1:
        _, p = rd_vu(b, p)
    elif ref == 2:
        n, p = rd_vu(b, p)
        for _ in range(n):
            p = _skip_str(b, p)
    elif ref in (3, 4, 5):
        p = _skip_str(b, p)
    elif ref == 6:
        p = _skip_str(b, _skip_str(b, p))
    elif ref == 7:
        t, p = rd_vu(b, p)
        if t in (3, 5):
            p = _skip_str(b, p)
    elif ref == 8:
        n, p = rd_vu(b, p)
        for _ in range(n):
            p = _skip_any(b, p)
    elif ref == 9:
        p = _skip_any(b, _skip_str(b, p))
    return p


def read_ds(b, p):
    n, p = rd_vu(b, p)
    out = []
    for _ in range(n):
        c, p = rd_vu(b, p)
        k, p = rd_vu(b, p)
        rs = []
        for _ in range(k):
            a, p = rd_vu(b, p)
            l, p = rd_vu(b, p)
            rs.append((a, l))
        out.append((c, rs))
    return out, p


def encode_ds(ds):
    o = bytearray(vu(len(ds)))
    for c, rs in ds:
        o += vu(c) + vu(len(rs))
        for a, l in rs:
            o += vu(a) + vu(l)
    return bytes(o)
