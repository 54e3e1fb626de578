"""Synthetic RNA pairs from a counter-based splitmix64 stream.

The same generator exists in C (`oracle/sed_oracle.c: sed_synth_seq`) so that
every process — bench ranks, tests, the golden-fixture script — derives the
identical sequence for a pair index without shipping data around.

Definition (both languages):
    z_t   = mix64(seed64 + t * GAMMA),  t = 1, 2, ...       (splitmix64)
    seed64 = ((base + pair) << 1) | stream                   stream 0 = str1, 1 = str2
    symbol k = (z_{k//32 + 1} >> (2*(k % 32))) & 3  ->  "ACGU"[symbol]

For the "related" secondary set, str2 is str1 with each position mutated with
probability ~10% (a third splitmix stream decides mutate / new symbol).
"""
import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
BASE_SEED = 20261015
ALPHABET = "ACGU"


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * M1
    z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def stream_words(seed64, nwords):
    """nwords consecutive splitmix64 outputs for each seed (seed64: uint64 array)."""
    seed64 = np.asarray(seed64, dtype=np.uint64).reshape(-1, 1)
    t = np.arange(1, nwords + 1, dtype=np.uint64).reshape(1, -1)
    with np.errstate(over="ignore"):
        return _mix64(seed64 + t * GAMMA)


def pair_codes(pair_ids, length, stream, base=BASE_SEED):
    """uint8 codes (0..3 = A,C,G,U) of shape (len(pair_ids), length)."""
    pair_ids = np.asarray(pair_ids, dtype=np.uint64)
    seed64 = ((np.uint64(base) + pair_ids) << np.uint64(1)) | np.uint64(stream)
    nwords = (length + 31) // 32
    w = stream_words(seed64, nwords)                      # (P, nwords) uint64
    shifts = (np.arange(32, dtype=np.uint64) * np.uint64(2)).reshape(1, 1, 32)
    sym = (w[:, :, None] >> shifts) & np.uint64(3)        # (P, nwords, 32)
    return sym.reshape(len(pair_ids), nwords * 32)[:, :length].astype(np.uint8)


IUPAC = "AGCUYRWSKMDVHBN"


def iupac_codes(pair_ids, length, stream, base=BASE_SEED):
    """uint8 codes 0..14 (indices into IUPAC): 4-bit fields of the same stream, mod 15."""
    pair_ids = np.asarray(pair_ids, dtype=np.uint64)
    seed64 = ((np.uint64(base) + pair_ids) << np.uint64(1)) | np.uint64(stream)
    seed64 = seed64 ^ np.uint64(0x1F2E3D4C5B6A7988)
    nwords = (length + 15) // 16
    w = stream_words(seed64, nwords)
    shifts = (np.arange(16, dtype=np.uint64) * np.uint64(4)).reshape(1, 1, 16)
    sym = ((w[:, :, None] >> shifts) & np.uint64(15)) % np.uint64(15)
    return sym.reshape(len(pair_ids), nwords * 16)[:, :length].astype(np.uint8)


def lengths(pair_ids, lo, hi, stream=2, base=BASE_SEED):
    """Per-id lengths uniform in [lo, hi] (for ragged workloads such as all-vs-all)."""
    pair_ids = np.asarray(pair_ids, dtype=np.uint64)
    seed64 = ((np.uint64(base) + pair_ids) << np.uint64(1)) | np.uint64(stream & 1)
    seed64 = seed64 ^ np.uint64(0xA5A5A5A5DEADBEEF + stream)
    w = stream_words(seed64, 1)[:, 0]
    return (lo + (w % np.uint64(hi - lo + 1))).astype(np.int32)


def pair_strings(pair_id, n, m, base=BASE_SEED):
    """(str1, str2) for one synthetic pair, as ACGU text."""
    lut = np.frombuffer(ALPHABET.encode(), dtype=np.uint8)
    a = lut[pair_codes([pair_id], n, 0, base)[0]].tobytes().decode()
    b = lut[pair_codes([pair_id], m, 1, base)[0]].tobytes().decode()
    return a, b


def related_codes(pair_ids, length, rate_per_256=26, base=BASE_SEED):
    """str1 codes and a mutated copy (substitutions only, ~10%)."""
    a = pair_codes(pair_ids, length, 0, base)
    pair_ids = np.asarray(pair_ids, dtype=np.uint64)
    seed64 = ((np.uint64(base) + pair_ids) << np.uint64(1)) | np.uint64(1)
    seed64 = seed64 ^ np.uint64(0x5DEECE66D)
    w = stream_words(seed64, (length + 3) // 4)           # 16 bits per position
    sh = (np.arange(4, dtype=np.uint64) * np.uint64(16)).reshape(1, 1, 4)
    r = ((w[:, :, None] >> sh) & np.uint64(0xFFFF)).reshape(len(pair_ids), -1)[:, :length]
    mutate = (r & np.uint64(0xFF)) < np.uint64(rate_per_256)
    new = ((r >> np.uint64(8)) & np.uint64(3)).astype(np.uint8)
    b = np.where(mutate, new, a).astype(np.uint8)
    return a, b
