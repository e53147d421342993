"""Pure-Python restatement of NeuroKmer's hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as a checker.  It is an independent second restatement of
the reference (written separately from oracle/nk_oracle.c) used to generate the
committed golden fixtures under tests/golden/ and to cross-check the C oracle.
Pure-Python loops: small inputs only.

Reference lines restated (MrObadiahEJ/NeuroKmer):
  src/models.rs:34-51         LifNeuron::update (f32, two roundings, never fused)
  src/models.rs:145-173       EnergyTracker
  src/models.rs:186-269       RollingKmerHash new/init/slide (release-mode u64)
  src/utils.rs:26-39          pack_kmer
  src/spiking_hash.rs:78-82   map_kmer_to_neuron = SipHasher13(0,0) over u64 LE % pool
  src/spiking_hash.rs:84-201  process_parallel
  src/spiking_hash.rs:277-486, 544-659  process_file_streaming (+AVX2 LIF)
  src/spiking_hash.rs:661-673 top_abundant_neurons
  src/main.rs:49-74           CLI result block
"""
from __future__ import annotations

import struct

M64 = (1 << 64) - 1


# ---------------------------------------------------------------- SipHash ---
def _rotl(x: int, b: int) -> int:
    return ((x << b) | (x >> (64 - b))) & M64


def siphash(c_rounds: int, d_rounds: int, k0: int, k1: int, msg: bytes) -> int:
    """SipHash-c-d (siphasher 1.0.2 semantics, Cargo.lock:1520-1522)."""
    v = [0x736F6D6570736575 ^ k0, 0x646F72616E646F6D ^ k1,
         0x6C7967656E657261 ^ k0, 0x7465646279746573 ^ k1]

    def rnd():
        v[0] = (v[0] + v[1]) & M64; v[1] = _rotl(v[1], 13); v[1] ^= v[0]; v[0] = _rotl(v[0], 32)
        v[2] = (v[2] + v[3]) & M64; v[3] = _rotl(v[3], 16); v[3] ^= v[2]
        v[0] = (v[0] + v[3]) & M64; v[3] = _rotl(v[3], 21); v[3] ^= v[0]
        v[2] = (v[2] + v[1]) & M64; v[1] = _rotl(v[1], 17); v[1] ^= v[2]; v[2] = _rotl(v[2], 32)

    n = len(msg)
    full = n - (n % 8)
    for i in range(0, full, 8):
        m = int.from_bytes(msg[i:i + 8], "little")
        v[3] ^= m
        for _ in range(c_rounds):
            rnd()
        v[0] ^= m
    b = ((n & 0xFF) << 56) | int.from_bytes(msg[full:], "little")
    v[3] ^= b
    for _ in range(c_rounds):
        rnd()
    v[0] ^= b
    v[2] ^= 0xFF
    for _ in range(d_rounds):
        rnd()
    return v[0] ^ v[1] ^ v[2] ^ v[3]


def sip13_u64(m: int) -> int:
    """SipHasher13::new_with_keys(0,0); u64::hash (write_u64: 8 LE bytes); finish()."""
    return siphash(1, 3, 0, 0, (m & M64).to_bytes(8, "little"))


def map_kmer_to_neuron(kmer: int, pool: int) -> int:
    """src/spiking_hash.rs:78-82"""
    return sip13_u64(kmer) % pool


# ----------------------------------------------------------- k-mer keys ---
_FWD = {ord(c): v for c, v in zip("ACGTacgt", [0, 1, 2, 3, 0, 1, 2, 3])}
_CMP = {ord(c): v for c, v in zip("ACGTacgt", [3, 2, 1, 0, 3, 2, 1, 0])}


class RollingKmerHash:
    """src/models.rs:175-299 with release-build integer semantics."""

    def __init__(self, k: int):
        self.k = k
        self.mask = ((1 << (2 * k)) - 1) if k < 32 else M64
        p = 1
        for _ in range(k - 1):
            p = (p << 2) & self.mask
        self.power = p
        self.fwd = 0
        self.rev = 0

    def init(self, first_k: bytes):
        assert len(first_k) == self.k, "Initialization slice length must equal k"
        self.fwd = 0
        for b in first_k:
            self.fwd = ((self.fwd << 2) & self.mask) | _FWD.get(b, 0)
        self.rev = 0
        for b in reversed(first_k):
            self.rev = ((self.rev << 2) & self.mask) | _CMP.get(b, 0)

    def slide(self, nxt: int, prev: int):
        self.fwd = (self.fwd - _FWD.get(prev, 0) * self.power) & M64
        self.fwd = (((self.fwd << 2) & M64) | _FWD.get(nxt, 0)) & self.mask
        sh = (2 * (self.k - 1)) & 63  # Rust release `<<` masks the shift amount
        self.rev = (self.rev >> 2) | ((_CMP.get(nxt, 0) << sh) & M64)
        self.rev &= self.mask

    def canonical(self) -> int:
        return min(self.fwd, self.rev)


def pack_kmer(window: bytes) -> int:
    """src/utils.rs:26-39: skips non-ACGT bytes; u64 keeps the last 32 bases."""
    packed = 0
    for b in window:
        if b in _FWD:
            packed = ((packed << 2) & M64) | _FWD[b]
    return packed


M128 = (1 << 128) - 1


def sip13_u128(key: int) -> int:
    """--kmer-width=128: SipHash-1-3 (key 0) over the u128's 16 LE bytes
    (Hasher::write_u128 -> to_ne_bytes on a little-endian host)."""
    return siphash(1, 3, 0, 0, (key & M128).to_bytes(16, "little"))


def kmer_keys128(seq: bytes, k: int, canonical: bool) -> list[int]:
    """--kmer-width=128 keys (the build's own mode), written per
    window rather than rolled, as an independent check of oracle/nk_oracle.c:
    fwd = sum code(b_i) << 2(k-1-i), rev = sum comp(b_i) << 2i, key = min;
    non-canonical: pack_kmer in 128 bits."""
    if not 1 <= k <= 64:
        raise ValueError("k must be in 1..64")
    out = []
    for i in range(0, len(seq) - k + 1):
        w = seq[i:i + k]
        if canonical:
            fwd = 0
            for b in w:
                fwd = (fwd << 2) | _FWD.get(b, 0)
            rev = 0
            for j, b in enumerate(w):
                rev |= _CMP.get(b, 0) << (2 * j)
            out.append(min(fwd, rev))
        else:
            packed = 0
            for b in w:
                if b in _FWD:
                    packed = ((packed << 2) & M128) | _FWD[b]
            out.append(packed)
    return out


def kmer_keys(seq: bytes, k: int, canonical: bool) -> list[int]:
    """The keys the reference derives from one record (src/spiking_hash.rs:102-138)."""
    if k <= 0:
        raise ValueError("k must be >= 1 (the reference panics)")
    out = []
    if canonical and len(seq) >= k:
        h = RollingKmerHash(k)
        h.init(seq[:k])
        out.append(h.canonical())
        for i in range(1, len(seq) - k + 1):
            h.slide(seq[i + k - 1], seq[i - 1])
            out.append(h.canonical())
    else:
        for i in range(0, len(seq) - k + 1):
            out.append(pack_kmer(seq[i:i + k]))
    return out


# -------------------------------------------------------------------- LIF ---
def f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def f32_bits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def lif_run(count: int, steps: int, thr: float, leak: float, refr: int,
            skip_zero: bool, v: float = 0.0, r: int = 0, spikes: int = 0):
    """`steps` calls of LifNeuron::update (src/models.rs:34-51) with
    c = (count as f64 / steps as f64) as f32.  Each f32 op is done in f64 and
    rounded to f32, which is exact for a single + or * of f32 operands."""
    total = float(count)
    if skip_zero and total == 0.0:
        return v, r, spikes
    c = f32(total / float(steps)) if steps else float("inf")
    thr = f32(thr)
    leak = f32(leak)
    for _ in range(steps):
        if r > 0:
            r -= 1
            continue
        v = f32(f32(v * leak) + c)
        if v >= thr:
            v = 0.0
            r = refr
            spikes += 1
    return v, r, spikes


# ---------------------------------------------------------------- counter ---
def _f64_as_u64(x: float) -> int:
    if not (x > 0.0):
        return 0
    if x >= 2.0 ** 64:
        return M64
    return int(x)


class SpikingKmerCounter:
    """src/spiking_hash.rs:16-77 (state), :84-201, :277-486, :661-695."""

    def __init__(self, k, threshold, leak, refractory, spike_cost, pool_size, use_canonical):
        self.k = k
        self.thr = threshold
        self.leak = leak
        self.refr = refractory
        self.cost = spike_cost
        self.pool = pool_size
        self.use_canonical = use_canonical
        self.steps = 1000
        self.v = [0.0] * pool_size
        self.r = [0] * pool_size
        self.sc = [0] * pool_size
        self.currents = [0] * pool_size
        self.kmer_per_neuron = [0] * pool_size
        self.counts: dict[int, int] = {}
        self.total_spikes = 0
        self.total_energy = 0

    def _add_spikes(self, n):
        self.total_spikes = (self.total_spikes + n) & M64
        self.total_energy = (self.total_energy + n * _f64_as_u64(self.cost * 1000.0)) & M64

    def _accumulate(self, seqs):
        cur = [0] * self.pool
        counts: dict[int, int] = {}
        for s in seqs:
            if len(s) < self.k and not self.use_canonical:
                continue
            for key in kmer_keys(s, self.k, self.use_canonical):
                counts[key] = (counts.get(key, 0) + 1) & 0xFFFFFFFF
                cur[map_kmer_to_neuron(key, self.pool)] += 1
        self.counts = counts
        self.kmer_per_neuron = [0] * self.pool
        for key in counts:
            self.kmer_per_neuron[map_kmer_to_neuron(key, self.pool)] += 1
        self.currents = cur

    def _lif_all(self, skip_zero):
        memo = {}
        total = 0
        for i in range(self.pool):
            st = (self.currents[i], self.v[i], self.r[i])
            if st not in memo:
                memo[st] = lif_run(self.currents[i], self.steps, self.thr, self.leak,
                                   self.refr, skip_zero, self.v[i], self.r[i], 0)
            v, r, n = memo[st]
            self.v[i], self.r[i] = v, r
            self.sc[i] += n
            total += n
        return total

    def process_parallel(self, seqs):
        self._accumulate(seqs)
        self._add_spikes(self._lif_all(skip_zero=True))

    def process_streaming(self, seqs):
        self._accumulate(seqs)
        self.simulate_spikes_auto()  # src/spiking_hash.rs:482

    def simulate_spikes_auto(self):
        """:697-714 -> simulate_spikes_simd (:544-659): every neuron, zero
        current included, from the held currents; steps == 0 returns first."""
        if self.steps == 0:
            return
        self._add_spikes(self._lif_all(skip_zero=False))

    def top_abundant_neurons(self, n):
        order = sorted(range(self.pool), key=lambda i: -self.sc[i])  # stable
        return [(i, self.sc[i], self.kmer_per_neuron[i]) for i in order[:n]]

    def get_count(self, kmer):
        return self.counts.get(kmer)

    def energy_used(self):
        return self.total_energy / 1000.0


# ------------------------------------------------------------ CLI output ---
def rust_f64_display(x: float) -> str:
    """Rust `{}` for f64: shortest round-trip digits, never exponent form."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "inf" if x > 0 else "-inf"
    r = repr(float(x))
    if "e" in r or "E" in r:
        mant, exp = r.lower().split("e")
        exp = int(exp)
        neg = mant.startswith("-")
        mant = mant.lstrip("-")
        if "." in mant:
            ip, fp = mant.split(".")
        else:
            ip, fp = mant, ""
        digits = (ip + fp).lstrip("0") or "0"
        point = len(ip) + exp
        if point <= 0:
            s = "0." + "0" * (-point) + digits
        elif point >= len(ip + fp):
            s = (ip + fp) + "0" * (point - len(ip + fp))
        else:
            s = (ip + fp)[:point] + "." + (ip + fp)[point:]
        s = s.lstrip("0") or "0"
        if s.startswith("."):
            s = "0" + s
        return ("-" if neg else "") + s
    if r.endswith(".0"):
        r = r[:-2]
    return r


def cli_result_block(counter: SpikingKmerCounter, pool_size: int, streaming: bool) -> str:
    """The stdout block printed by src/main.rs:49-74."""
    lines = ["", "=== Top 20 Abundant Neuron Groups (Highest Spike Rates) ==="]
    top = counter.top_abundant_neurons(20)
    if not top:
        lines.append("No spikes fired (empty file or too small k)")
    else:
        for rank, (idx, spikes, uniques) in enumerate(top):
            lines.append(f"{rank + 1:3}: Neuron {idx:6} → {spikes:8} spikes "
                         f"({uniques} unique k-mers colliding)")
    lines.append("")
    lines.append(f"Total spikes fired: {counter.total_spikes}")
    lines.append(f"Simulated energy used: {rust_f64_display(counter.energy_used())}")
    lines.append(f"Neuron pool size used: {pool_size}")
    lines.append(f"Streaming mode: {'true' if streaming else 'false'}")
    return "\n".join(lines) + "\n"
