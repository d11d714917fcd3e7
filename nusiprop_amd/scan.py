"""Parameter-scan grids and their partition over GPUs.

Scan points are independent propagations (one calculate_flux::evolve() each),
so a multi-GPU scan is a pure partition: contiguous blocks of the flattened
grid per rank, no collective on the data path; results are gathered on the
host at the end.  Points that share (mphi, g, mntot, flags,
grid) also share their Stage-A tables (nuSIprop.hpp:217-253 do not depend on
si or norm), so the partition keeps such groups whole (shard_aligned).
"""
import numpy as np

BASE = dict(mntot=0.1, norm=1.0, majorana=True, non_resonant=True, normal_ordering=True, flav=2, phiphi=False,
            source_model=1, N_bins_E=300, lEmin=12.0, lEmax=17.0, zmax=5.0)

# BASELINE config 1: test.cpp:6-23 (N_E = 100, lE 9 -> 14, the fork's DSNB source, phi-phi off)
C1 = dict(mphi=6e5, g=0.01, mntot=0.1, si=2.5, norm=6.0, majorana=True, non_resonant=True, normal_ordering=True,
          N_bins_E=100, lEmin=9.0, lEmax=14.0, zmax=5.0, flav=2, phiphi=False, source_model=0)


def c4_points(si=2.5, n_mphi=32, n_g=32, **over):
    """BASELINE config 4: mphi in logspace(5.5, 8, 32) x g in logspace(-3, 0, 32), gamma = 2.5, power law."""
    base = dict(BASE, **over)
    return [dict(base, mphi=float(m), g=float(g), si=float(si))
            for m in np.logspace(5.5, 8.0, n_mphi) for g in np.logspace(-3.0, 0.0, n_g)]


def c4s_points(si=2.5, n_mphi=32, n_g=32, step=4, **over):
    """The opt-in shift-reuse scan (NUSI_OPT_SHIFT_REUSE): C4's g grid and 32 m_phi on the
    lattice m_max r^(-o/2), o = 0, step, 2 step, ... (r = 10^((lEmax - lEmin) / N_E), the table axis' bin ratio),
    m_max = 10^6.533 (o = 124 reaches 10^5.5, C4's lower end).  Needs K >= step (n_mphi - 1)."""
    base = dict(BASE, **over)
    r = 10 ** ((base["lEmax"] - base["lEmin"]) / base["N_bins_E"])
    m_max = 10 ** 6.533
    return [dict(base, mphi=float(m_max * r ** (-step * k / 2)), g=float(g), si=float(si))
            for k in range(n_mphi) for g in np.logspace(-3.0, 0.0, n_g)]


def c5_points(**over):
    """BASELINE config 5: mphi (64) x g (64) x gamma in linspace(2, 3, 16) = 65 536 points, gamma fastest."""
    base = dict(BASE, **over)
    return [dict(base, mphi=float(m), g=float(g), si=float(s))
            for m in np.logspace(5.5, 8.0, 64) for g in np.logspace(-3.0, 0.0, 64) for s in np.linspace(2.0, 3.0, 16)]


def shard(n_points, world, rank):
    """Contiguous block [lo, hi) of rank `rank` (sizes differ by at most one)."""
    q, r = divmod(n_points, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


TABLE_KEYS = ("mphi", "g", "mntot", "majorana", "non_resonant", "normal_ordering", "flav", "phiphi",
              "N_bins_E", "lEmin", "lEmax", "zmax")


def table_key(p):
    """The fields a point's Stage-A tables depend on (nuSIprop.hpp:217-253 read neither si, norm nor the
    source): points with equal keys share one table on a GPU (nusi_plan_evolve deduplicates them)."""
    return tuple(p.get(k) for k in TABLE_KEYS)


def group_bounds(points):
    """Start index of every maximal run of consecutive points sharing a table key, plus len(points)."""
    b = [0]
    for i in range(1, len(points)):
        if table_key(points[i]) != table_key(points[i - 1]):
            b.append(i)
    if points:
        b.append(len(points))
    return b


def shard_aligned(points, world, rank):
    """Contiguous block [lo, hi) of rank `rank` whose ends fall on table-group boundaries where that costs
    little balance (runs of points sharing a table stay on one GPU): each end is the group
    boundary nearest to the even split r * n / world, unless that boundary is more than half a block away
    -- a group much larger than n / world (e.g. a pure spectral-index scan: one table) -- in which case the
    cut is the even split itself and the group's table is built on both ranks (one Stage-A table per GPU is
    cheaper than idle GPUs)."""
    n = len(points)
    if n == 0:
        return 0, 0
    b = group_bounds(points)
    tol = n / world / 2.0

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return n
        ideal = r * n / world
        near = min(b, key=lambda x: (abs(x - ideal), x))
        return near if abs(near - ideal) <= tol else int(round(ideal))

    return cut(rank), max(cut(rank), cut(rank + 1))


def cascade_bytes_per_point(N, Nz):
    """Algorithmic HBM bytes of one propagation's cascade:
    8 * [ (Nz-1) N(N-1)/2 alpha reads + 6 N (Nz-1) Gamma/alphaTilde/flux terms + Nz N ]."""
    return 8 * ((Nz - 1) * N * (N - 1) // 2 + 6 * N * (Nz - 1) + Nz * N)


WSP_NJ, WSP_RT = 16, 8   # the step-pass instance k_cascade_bs<16, 1, 1, 8, 1>: step slots per pass, 16-row tiles per push wave


def cascade_passes(N, Nz, nj=None):
    """The step-pass cascade's passes: (first step slot jb, stages Ts, column of local stage 0 c0); nj steps per pass
    (default the step-pass kernel's, GB_NJ for the gamma batch)."""
    nj = nj or WSP_NJ
    T, nst = N + Nz - 2, Nz - 1
    return [(jb, N - 1 + min(nj, nst - jb), T - 1 - jb) for jb in range(0, nst, nj)]


GB_NJ, GB_RT = 6, 2   # the gamma batch k_cascade_bs<6, 16, 1, 2, 2>: steps per pass, 16-row tiles per push wave


def gamma_batches(points, rhs=16):
    """The gamma-batch workgroups nusi_plan_evolve forms (NUSI_OPT_CASCADE_RHS = rhs >= 3): per table, its
    power-law points in near-equal batches of <= rhs when there are at least 3.  Returns the batch sizes."""
    from collections import Counter
    cnt = Counter(table_key(p) for p in points if p.get("source_model", 0) == 1)
    out = []
    for c in cnt.values():
        if c >= 3:
            nb = -(-c // rhs)
            out += [c * (k + 1) // nb - c * k // nb for k in range(nb)]
    return out


def bs_groups(points, rhs=0, gamma=True, pairs=True):
    """The workgroups of the block-synchronous cascade as nusi_plan_evolve forms them (nusi_capi.cpp, the k_cascade_bs
    grouping): per table, all its points (any source) in near-equal groups of up to min(rhs or 16, 16) when it has 3
    or more and the gamma instance fits the grid (`gamma`), else pairs when it has 2 (`pairs`), else one per
    workgroup; a group of 3+ runs on k_cascade_bs_gamma, of 2 on k_cascade_bs_pairs, of 1 on k_cascade_bs.
    Returns the group sizes."""
    from collections import Counter
    rmax = rhs or 16
    g16, g2 = gamma and rmax >= 3, pairs and rmax >= 2
    out = []
    for c in Counter(table_key(p) for p in points).values():
        cap = min(rmax, 16) if (g16 and c >= 3) else 2 if (g2 and c >= 2) else 1
        nb = -(-c // cap)
        out += [c * (k + 1) // nb - c * k // nb for k in range(nb)]
    return out


def cascade_gb_bytes_per_batch(N, Nz):
    """HBM bytes one gamma-batch workgroup must read: the columns each pass visits (as the step-pass kernel), Gamma
    and alphaTilde; the FIFO of the passes' last step stays in L2/MALL (3 N x 16 doubles per pass, written once,
    read once) and the fluxes are counted per point (6 N x 8 B)."""
    T = N + Nz - 2
    cols = 0
    for jb, Ts, c0 in cascade_passes(N, Nz, GB_NJ):
        lo = max(1, c0 + 1 - 4 * ((Ts - 1) // 4))
        cols += sum(range(lo, min(c0 + 1, T - 1) + 1))
    return 8 * (cols + 2 * T)


def cascade_gb_flops_per_batch(N, Nz):
    """fp64 matrix-core flops one gamma-batch workgroup issues: per pass and block q >= 1, one v_mfma_f64_16x16x4f64
    (16 rows x 16 points x 4 columns, 2048 flops) per row tile below r = c0 - 4q and per step tile (GB_NJ)."""
    T = N + Nz - 2
    ntile = -(-(T - 1) // (16 * GB_RT)) * GB_RT
    tiles = sum(min(ntile, -(-(c0 - 4 * q) // 16)) for jb, Ts, c0 in cascade_passes(N, Nz, GB_NJ)
                for q in range(1, (Ts - 1) // 4 + 1) if c0 - 4 * q > 0)
    return tiles * GB_NJ * 2 * 16 * 16 * 4


def cascade_min_bytes_per_point(N, Nz, passes=False):
    """HBM bytes the wavefront cascade must move per propagation: each alpha column of the
    packed table once (T(T-1)/2), Gamma and alphaTilde (2T), both flux outputs (6N).  With step
    passes (Nz - 1 > 48) every pass reads the columns its stages visit (column c holds c entries)."""
    T = N + Nz - 2
    if not passes:
        return 8 * (T * (T - 1) // 2 + 2 * T + 6 * N)
    cols = 0
    for jb, Ts, c0 in cascade_passes(N, Nz):
        lo = max(1, c0 + 1 - 4 * ((Ts - 1) // 4))
        cols += sum(range(lo, min(c0 + 1, T - 1) + 1))
    return 8 * (cols + 2 * T + 6 * N)


def cascade_mfma_flops_per_point(N, Nz):
    """fp64 matrix-core flops the MFMA-push cascade (k_cascade_bs, one point per workgroup) issues per propagation: block q
    (stage 4q, q >= 1) runs one v_mfma_f64_16x16x4f64 (2*16*16*4 flops) per 16-row tile starting below
    r = T-1-4q, per 16-step tile (NJ/16 of them, NJ = Nz-1 rounded up to 16/32/48).  Grids with more
    steps run the step-pass instance: the same count per pass, one step tile."""
    T, n = N + Nz - 2, Nz - 1
    NJ = 16 if n <= 16 else 32 if n <= 32 else 48 if n <= 48 else 0
    waves = (T - 1 + 63) // 64
    if not NJ and T >= 2:   # the step-pass kernel: one 16-step tile, RT row tiles per push wave
        ntile = -(-(T - 1) // (16 * WSP_RT)) * WSP_RT
        tiles = sum(min(ntile, -(-(c0 - 4 * q) // 16)) for jb, Ts, c0 in cascade_passes(N, Nz)
                    for q in range(1, (Ts - 1) // 4 + 1) if c0 - 4 * q > 0)
        return tiles * 2 * 16 * 16 * 4
    if not NJ or T < 2 or waves * 64 + 64 > 512:
        return 0
    tiles = sum(min(4 * waves, -(-(T - 1 - 4 * q) // 16)) for q in range(1, (T - 1) // 4 + 1) if T - 1 - 4 * q > 0)
    return tiles * (NJ // 16) * 2 * 16 * 16 * 4


def alpha_entries_per_point(N, Nz):
    """Stage-A alpha entries per propagation, T(T-1)/2 with T = N + Nz - 2 (each summed over 3 mass states)."""
    T = N + Nz - 2
    return T * (T - 1) // 2
