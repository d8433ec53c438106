"""Vectorised numpy restatement of the ChaCha20 block function (RFC 8439 section 2.3) with the
library's 64-bit counter / 64-bit nonce layout (csrc/chacha.h), and of the three samplers built
on it (csrc/ckks.hip: uniform, centered binomial, ternary).  Test infrastructure only: the GPU
tests compare the device samplers with these, and the CPU tests pin this file to the RFC's
known-answer vectors."""
import numpy as np

_CONST = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)


def _rotl(x, r):
    return ((x << np.uint32(r)) | (x >> np.uint32(32 - r))).astype(np.uint32)


def blocks(key, counters, nonce):
    """key: 8 uint32 words; counters: array of block counters; returns [len(counters), 16] uint32."""
    counters = np.asarray(counters, dtype=np.uint64)
    m = counters.size
    st = np.empty((16, m), dtype=np.uint32)
    st[0:4] = _CONST[:, None]
    st[4:12] = np.asarray(key, dtype=np.uint32)[:, None]
    st[12] = (counters & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    st[13] = (counters >> np.uint64(32)).astype(np.uint32)
    st[14] = np.uint32(nonce & 0xFFFFFFFF)
    st[15] = np.uint32(nonce >> 32)
    x = st.copy()

    def qr(a, b, c, d):
        with np.errstate(over="ignore"):
            x[a] += x[b]; x[d] = _rotl(x[d] ^ x[a], 16)
            x[c] += x[d]; x[b] = _rotl(x[b] ^ x[c], 12)
            x[a] += x[b]; x[d] = _rotl(x[d] ^ x[a], 8)
            x[c] += x[d]; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    with np.errstate(over="ignore"):
        out = x + st
    return out.T.copy()


def words64(key, nblocks, nonce):
    """The first 8 * nblocks 64-bit keystream words of draw `nonce`."""
    b = blocks(key, np.arange(nblocks, dtype=np.uint64), nonce).astype(np.uint64)
    return (b[:, 0::2] | (b[:, 1::2] << np.uint64(32))).reshape(-1)


def sample_uniform(key, nonce, moduli, n):
    """[L][n] residues: element e takes 128-bit word pair e, reduced mod q (ckks.hip uniform_kernel)."""
    L = len(moduli)
    w = words64(key, n * L // 4, nonce)
    lo, hi = w[0::2], w[1::2]
    out = np.empty(n * L, dtype=np.uint64)
    for l, q in enumerate(moduli):
        s = slice(l * n, (l + 1) * n)
        out[s] = [((int(h) << 64) | int(o)) % q for h, o in zip(hi[s], lo[s])]
    return out


def _small(key, nonce, n):
    return words64(key, n // 8, nonce)


def sample_cbd(key, nonce, moduli, n):
    w = _small(key, nonce, n)
    m21 = np.uint64(0x1FFFFF)
    pc = np.vectorize(lambda v: bin(int(v)).count("1"), otypes=[np.int64])
    v = pc(w & m21) - pc((w >> np.uint64(21)) & m21)
    return np.concatenate([np.where(v >= 0, v, v + q).astype(np.uint64) for q in moduli])


def sample_ternary(key, nonce, moduli, n):
    w = _small(key, nonce, n)
    v = (w % np.uint64(3)).astype(np.int64) - 1
    return np.concatenate([np.where(v >= 0, v, v + q).astype(np.uint64) for q in moduli])
