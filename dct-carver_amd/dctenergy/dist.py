"""Row-band sharding of one frame over ranks (one process per GPU).

Rank k of G owns global rows [Y0, Y1) of a frame of height H.  An output row
y reads input rows y-(N/2-1) .. y+N/2 (src/render.c:146-152; replicate clamp
at the *global* image border), so a band needs hl = N/2-1 rows from the rank
above (its top halo) and hr = N/2 rows from the rank below (its bottom halo).
Those rows are the only bytes that cross ranks: one point-to-point exchange
per frame (RCCL over xGMI with backend "nccl"; gloo on CPU in tests).

The band buffer holds [top halo | own rows | bottom halo] contiguously, so the
kernel addresses it as global rows [Y0 - top, Y1 + bot).
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Band:
    rank: int
    world: int
    H: int          # global frame height
    Y0: int         # own rows [Y0, Y1)
    Y1: int
    hl: int         # N/2 - 1
    hr: int         # N/2

    @property
    def own(self):
        return self.Y1 - self.Y0

    @property
    def top(self):
        """halo rows held above Y0 (none at the global top)"""
        return self.hl if self.rank > 0 else 0

    @property
    def bot(self):
        """halo rows held below Y1 (none at the global bottom)"""
        return self.hr if self.rank < self.world - 1 else 0

    @property
    def rows(self):
        return self.top + self.own + self.bot

    @property
    def row0(self):
        """global row index of buffer row 0"""
        return self.Y0 - self.top

    def interior(self):
        """output rows computable from own rows alone (before the halos land)"""
        return self.Y0 + self.top, self.Y1 - self.bot

    def edges(self):
        """output row ranges that need a halo"""
        out = []
        if self.top:
            out.append((self.Y0, self.Y0 + self.top))
        if self.bot:
            out.append((self.Y1 - self.bot, self.Y1))
        return out


def make_band(H, rank, world, n, rows_per_rank=None):
    """Band of `rank`.  rows_per_rank=None splits H evenly (strong scaling);
    otherwise every rank owns rows_per_rank rows of a frame of height
    world * rows_per_rank (weak scaling)."""
    if rows_per_rank is None:
        Y0, Y1 = H * rank // world, H * (rank + 1) // world
    else:
        if H != world * rows_per_rank:
            raise ValueError("weak scaling: H must be world * rows_per_rank")
        Y0, Y1 = rank * rows_per_rank, (rank + 1) * rows_per_rank
    band = Band(rank, world, H, Y0, Y1, n // 2 - 1, n // 2)
    if world > 1 and band.own < band.hr:
        raise ValueError(f"every rank needs >= {band.hr} rows (N={n})")
    return band


def rccl_log_setup(tag="dcte"):
    """Before init_process_group (backend "nccl" = RCCL): have RCCL write its
    INFO log (connection set-up included) to a per-process file, so the run
    can report which transport actually carried the halos
    (transport_summary).  A level the caller set below INFO (unset, VERSION,
    WARN -- the GPU boxes export NCCL_DEBUG=VERSION) is raised to INFO; the
    log goes to the file, not to the caller's streams.  Returns the file path,
    or None when the caller already routes RCCL's log (NCCL_DEBUG_FILE) or
    asked for more than INFO."""
    import os
    import tempfile
    level = os.environ.get("NCCL_DEBUG", "").upper()
    if os.environ.get("NCCL_DEBUG_FILE") or level in ("INFO", "TRACE"):
        return None
    path = os.path.join(tempfile.gettempdir(), f"{tag}.rccl.{os.getpid()}.log")
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,P2P,NET"
    os.environ["NCCL_DEBUG_FILE"] = path
    return path


def transport_summary(path, rank=None):
    """What RCCL's INFO log says about this rank's connections: every
    "a[..] -> b[..] via TRANSPORT" line, counted per (peer, transport) -- e.g.
    P2P/IPC (xGMI peer-to-peer), SHM, NET/Socket (the one-GPU rehearsal's
    loopback) -- and the RCCL version line."""
    import re
    out = {"connections": {}, "version": None, "log": path}
    try:
        with open(path, errors="replace") as f:
            text = f.read()
    except OSError:
        out["error"] = "no RCCL log"
        return out
    m = re.search(r"(?:RCCL|NCCL) version[ :]*([\w.+-]+)", text)
    out["version"] = m.group(1) if m else None
    pat = re.compile(r"(\d+)\[[^\]]*\] -> (\d+)\[[^\]]*\][^\n]*? via ([^\s,]+)")
    conns = {}
    for a, b, via in pat.findall(text):
        if rank is not None and int(a) != rank and int(b) != rank:
            continue
        key = f"{a}->{b} {via}"
        conns[key] = conns.get(key, 0) + 1
    out["connections"] = conns
    out["transports"] = sorted({k.split(" ", 1)[1] for k in conns})
    return out


def halo_ops(buf, band, group=None):
    """P2P ops that fill `buf`'s halo rows from the neighbour ranks and send
    this rank's edge rows to them (buf: [band.rows, ...] contiguous tensor).

    rank k-1's bottom halo = my first hr own rows; rank k+1's top halo = my
    last hl own rows."""
    import torch.distributed as dist
    ops = []
    k, G = band.rank, band.world
    t, own = band.top, band.own
    if k > 0:
        if band.hl:
            ops.append(dist.P2POp(dist.irecv, buf[:t], k - 1, group))
        ops.append(dist.P2POp(dist.isend, buf[t:t + band.hr], k - 1, group))
    if k < G - 1:
        ops.append(dist.P2POp(dist.irecv, buf[t + own:], k + 1, group))
        if band.hl:
            ops.append(dist.P2POp(dist.isend, buf[t + own - band.hl:t + own], k + 1, group))
    return ops


def exchange_halos(buf, band, group=None):
    """Start the halo exchange; returns the request list (empty at world 1)."""
    import torch.distributed as dist
    ops = halo_ops(buf, band, group)
    if not ops:
        return []
    return dist.batch_isend_irecv(ops)


def global_minmax(minmax, group=None):
    """Frame-wide {min, max} from every rank's band {min, max} (a 2-float
    tensor, e.g. from dcte_minmax_device), in place: ONE all-reduce of
    [min, -max] with MIN (negation is exact)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return minmax
    minmax[1:2].neg_()
    dist.all_reduce(minmax, op=dist.ReduceOp.MIN, group=group)
    minmax[1:2].neg_()
    return minmax


def energy_image_u8(ctx, band_map, out_u8, mode, channels=1, device=0, group=None):
    """This rank's rows of the 8-bit energy layer of a row-sharded frame
    (display_carver_energy, src/render.c:175-202, on a frame split over
    ranks): band min/max on the device, one all-reduce of 2 floats, then the
    band normalised with the frame-wide min/max -- the same bytes the single-
    device dcte_energy_image_u8 writes for those rows.
    band_map: contiguous float32 CUDA tensor (own rows); out_u8: its
    uint8 tensor (x channels)."""
    import torch
    if not band_map.is_contiguous() or not out_u8.is_contiguous():
        raise ValueError("band_map and out_u8 must be contiguous")
    mm = torch.empty(2, dtype=torch.float32, device=band_map.device)
    stream = torch.cuda.current_stream(band_map.device).cuda_stream
    ctx.minmax_device(band_map.data_ptr(), band_map.numel(), mm.data_ptr(), stream, device)
    global_minmax(mm, group)
    ctx.normalize_u8_device(band_map.data_ptr(), band_map.numel(), mm.data_ptr(),
                            out_u8.data_ptr(), mode, channels, stream, device)
    return out_u8


def band_rows(H, k, world):
    """Own rows [Y0, Y1) of rank k for an even split of H rows (make_band's
    strong split; equal to the weak split when H = world * rows_per_rank)."""
    return H * k // world, H * (k + 1) // world


def gather_bands(part, band, dst=0, group=None):
    """Every rank's own rows -> the whole frame on rank `dst`;
    None on the other ranks.  Bands are padded to ceil(H / world) rows so one
    gather moves them (RCCL: one send per rank over its xGMI link)."""
    import torch
    import torch.distributed as dist
    tall = -(-band.H // band.world)
    pad = part.new_zeros((tall,) + tuple(part.shape[1:]))
    pad[:band.own] = part
    bufs = [torch.empty_like(pad) for _ in range(band.world)] if band.rank == dst else None
    dist.gather(pad, bufs, dst=dst, group=group)
    if band.rank != dst:
        return None
    return torch.cat([bufs[k][:b - a] for k, (a, b) in
                      enumerate(band_rows(band.H, k, band.world) for k in range(band.world))])
