"""Chromosome sharding across GPUs and the gather of per-chromosome record streams.

SCCG compresses one chromosome pair per invocation and pairs are independent,
so the multi-GPU job is: LPT-assign pairs to ranks (largest target first onto the least-loaded
rank), compress locally, then move every rank's record texts to rank 0 -- the job's only data
exchange -- with one all-gather of the int64 sizes and one gather of the (max-size) packed streams
to rank 0 only (RCCL over xGMI with the "nccl" backend on GPUs; "gloo" on CPU for tests).
"""
from __future__ import annotations

import heapq

import torch
import torch.distributed as dist


# UCSC chromInfo lengths: chr1..22, X, Y.  hg18 = reference, hg19 = target.
CHROMS = [f"chr{i}" for i in range(1, 23)] + ["chrX", "chrY"]
HG18 = [247249719, 242951149, 199501827, 191273063, 180857866, 170899992, 158821424, 146274826, 140273252,
        135374737, 134452384, 132349534, 114142980, 106368585, 100338915, 88827254, 78774742, 76117153,
        63811651, 62435964, 46944323, 49691432, 154913754, 57772954]
HG19 = [249250621, 243199373, 198022430, 191154276, 180915260, 171115067, 159138663, 146364022, 141213431,
        135534747, 135006516, 133851895, 115169878, 107349540, 102531392, 90354753, 81195210, 78077248,
        59128983, 63025520, 48129895, 51304566, 155270560, 59373566]


def lpt_shard(sizes: list[int], world: int) -> list[list[int]]:
    """Longest-processing-time-first: item indices per rank, each rank's list in input order."""
    if world < 1:
        raise ValueError("world must be >= 1")
    heap = [(0, r) for r in range(world)]
    out: list[list[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + sizes[i], r))
    return [sorted(x) for x in out]


def max_over_mean(sizes: list[int], world: int) -> float:
    loads = [sum(sizes[i] for i in part) for part in lpt_shard(sizes, world)]
    return max(loads) / (sum(loads) / world) if sum(loads) else 1.0


def gather_to_root(buf: torch.Tensor, n: int, group=None) -> list[torch.Tensor] | None:
    """Gather the first `n` bytes of every rank's uint8 buffer `buf` to rank 0 (a gatherv).

    One all-gather of the int64 sizes (one host read of their max), then one gather of each rank's
    first max-size bytes straight out of `buf` (no staging copy unless `buf` is shorter than the
    largest part).  Only rank 0 receives.  Returns [part of rank r] (views, trimmed to the sizes)
    on rank 0 and None elsewhere.  `buf` lives on the device for RCCL, on the CPU for gloo."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = buf.device
    sz = torch.tensor([n], dtype=torch.int64, device=dev)
    sizes = [torch.empty(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, sz, group=group)
    sizes_h = torch.cat(sizes).cpu().tolist()
    mx = max(sizes_h) if sizes_h else 0
    if mx == 0:
        return [buf[:0] for _ in range(world)] if rank == 0 else None
    if buf.numel() >= mx:
        send = buf[:mx]
    else:
        send = torch.zeros(mx, dtype=torch.uint8, device=dev)
        send[:n] = buf[:n]
    parts = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(send, parts, dst=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    if rank != 0:
        return None
    return [parts[r][: sizes_h[r]] for r in range(world)]


class StreamGather:
    """The per-step gather of every rank's per-chromosome record streams to rank 0 with no host
    synchronisation inside the step and no padding (the genome job's only exchange,
    compression.cpp:584-610: one record file per pair).

    A stream's length is a function of its pair's inputs, so the lengths are exchanged once, in
    plan() (outside the timed region: one all_gather_object of {name: length}), and rank 0
    preallocates one receive tensor per remote stream of exactly that length.  step() then posts,
    in one batch_isend_irecv, one send per stream on the other ranks and the matching receives on
    rank 0 (RCCL point-to-point over xGMI on GPUs, gloo on CPU; both sides post in name order, so
    messages between two ranks match in order).  The only per-step check is on the host, against
    lengths the host already holds (the library returns each length synchronously): a stream whose
    length differs from the plan raises instead of being truncated.  Nothing is read back from the
    device, and the sends/receives are ordered behind the lanes' streams by stream waits
    (`after`), not by host syncs."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.plan_lengths: list[dict[str, int]] | None = None
        self.recv: dict[str, torch.Tensor] = {}
        self.local: dict[str, torch.Tensor] = {}

    def _peer(self, r: int) -> int:
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def plan(self, parts: dict[str, torch.Tensor], device: torch.device) -> None:
        """Exchange the per-stream lengths (outside the timed region) and allocate rank 0's
        receive tensors."""
        mine = {n: int(t.numel()) for n, t in parts.items()}
        got: list = [None] * self.world
        dist.all_gather_object(got, mine, group=self.group)
        self.plan_lengths = got
        if self.rank == 0:
            self.recv = {n: torch.empty(ln, dtype=torch.uint8, device=device)
                         for r in range(1, self.world) for n, ln in sorted(got[r].items())}

    def step(self, parts: dict[str, torch.Tensor], after=()) -> None:
        """Queue this step's gather.  `after`: CUDA streams the record tensors were written on
        (the current stream waits for them; nothing waits on the host)."""
        if self.plan_lengths is None:
            raise RuntimeError("StreamGather.step before plan()")
        mine = self.plan_lengths[self.rank]
        if set(parts) != set(mine):
            raise RuntimeError("StreamGather: the rank's chromosomes differ from the plan")
        for n, t in parts.items():
            if int(t.numel()) != mine[n]:
                raise RuntimeError(f"StreamGather: record stream {n} is {t.numel()} bytes, the plan has {mine[n]}: "
                                   "re-plan before the timed region")
        if torch.cuda.is_available():
            cur = torch.cuda.current_stream()
            for s in after:
                cur.wait_stream(s)
        self.local = dict(parts)
        ops = []
        if self.rank == 0:
            for r in range(1, self.world):
                for n in sorted(self.plan_lengths[r]):
                    if self.recv[n].numel():
                        ops.append(dist.P2POp(dist.irecv, self.recv[n], self._peer(r), self.group))
        else:
            for n in sorted(mine):
                if parts[n].numel():
                    ops.append(dist.P2POp(dist.isend, parts[n].reshape(-1), self._peer(0), self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()   # (RCCL: the current stream waits; gloo: the host, on CPU tensors)

    def result(self) -> dict[str, torch.Tensor] | None:
        """Rank 0: {name: record stream tensor} of every rank (after the step's work has run);
        None elsewhere."""
        if self.rank != 0:
            return None
        out = dict(self.local)
        out.update(self.recv)
        return out


def pack_records(parts: dict[str, bytes | torch.Tensor], device: torch.device) -> torch.Tensor:
    """One uint8 buffer: int64 header [n_names, len(names blob), len(blob_i)...], the NUL-joined
    names, then the blobs in name order."""
    names = sorted(parts)
    blobs = []
    for nme in names:
        v = parts[nme]
        if isinstance(v, torch.Tensor):
            blobs.append(v.to(device).reshape(-1))
        else:
            blobs.append(torch.frombuffer(bytearray(v), dtype=torch.uint8).to(device) if len(v)
                         else torch.zeros(0, dtype=torch.uint8, device=device))
    name_bytes = "\0".join(names).encode()
    head = torch.tensor([len(names), len(name_bytes)] + [int(b.numel()) for b in blobs], dtype=torch.int64)
    pieces = [head.view(torch.uint8).to(device)]
    if name_bytes:
        pieces.append(torch.frombuffer(bytearray(name_bytes), dtype=torch.uint8).to(device))
    return torch.cat(pieces + blobs)


def unpack_records(raw: bytes) -> dict[str, bytes]:
    """Inverse of pack_records."""
    import struct
    n_names, nb = struct.unpack_from("<qq", raw, 0)
    lens = struct.unpack_from(f"<{n_names}q", raw, 16)
    off = 16 + 8 * n_names
    names = raw[off: off + nb].decode().split("\0") if n_names else []
    off += nb
    out = {}
    for nme, ln in zip(names, lens):
        out[nme] = raw[off: off + ln]
        off += ln
    return out


def gather_records(parts: dict[str, bytes | torch.Tensor], device: torch.device | None = None,
                   group=None) -> dict[str, bytes] | None:
    """Gather {chromosome: record text} from every rank to rank 0 (pack_records + gather_to_root).

    `parts` values may be bytes or uint8 tensors (device tensors stay on the device for RCCL).
    Returns the merged dict on rank 0, None elsewhere."""
    dev = device or torch.device("cpu")
    buf = pack_records(parts, dev)
    got = gather_to_root(buf, int(buf.numel()), group=group)
    if got is None:
        return None
    merged: dict[str, bytes] = {}
    for part in got:
        merged.update(unpack_records(part.cpu().numpy().tobytes()))
    return merged


# -------------------------------------------------------------------------------------------------
# One chromosome's global walk split across ranks.
#
# The reference's global pass is ONE sequential walk over T' (compression.cpp:561, :64-161) with
# state (index, P = prev_match_end).  Two walks that reach the same state coincide afterwards, so
# the target can be cut into per-rank ranges exactly as the GPU walk cuts it into chunks:
#   1. rank r walks its range [h_r, h_{r+1}) from a guessed entry state (rank 0: the true start);
#   2. rounds: every rank's exit state goes to its successor (one all-gather of 2 int64 per rank);
#      a rank whose trajectory was not walked from its predecessor's current exit re-walks from it
#      and splices onto its old trajectory at the first common match (after a common match the
#      states are equal); the loop ends when no entry changed -- at most world - 1 rounds;
#   3. the per-rank match lists go to rank 0 (the record-stream gather of the genome job).
# The result is the single sequential walk exactly, whatever the guesses were.  `walker` is the
# per-rank engine: walker(x0, P0, x_end) -> (matches [(t, p, l)], (exit_x, exit_P)), the walk from
# state (x0, P0) until index >= x_end.
# -------------------------------------------------------------------------------------------------
def split_ranges(n_target: int, world: int) -> list[int]:
    """Range starts h_0 = 0 < ... < h_world = n_target (equal shares)."""
    return [n_target * r // world for r in range(world)] + [n_target]


def splice(new: list, old: list, new_exit: tuple, old_exit: tuple) -> tuple[list, tuple, bool]:
    """The re-walk `new` joined onto the old trajectory at their first common match: from there on
    the two walks coincide, so the old suffix (and exit) stand.  Returns (trajectory, exit, changed)."""
    pos = {m: i for i, m in enumerate(old)}
    for j, m in enumerate(new):
        i = pos.get(m)
        if i is not None:
            return new[:j] + old[i:], old_exit, False
    return new, new_exit, new_exit != old_exit


def split_walk(walker, n_target: int, guess_entry, group=None) -> list | None:
    """Run this rank's share of one chromosome's global walk and return the whole walk's match list
    on rank 0 (None elsewhere).  guess_entry(h) -> P: the speculative entry of a range starting at
    h (rank 0 uses the true start, P = -1)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    h = split_ranges(n_target, world)
    lo, hi = h[rank], h[rank + 1]
    entry = (0, -1) if rank == 0 else (lo, int(guess_entry(lo)))
    traj, exit_state = walker(entry[0], entry[1], hi)
    for _ in range(world):
        ex = torch.tensor([exit_state[0], exit_state[1]], dtype=torch.int64)
        exits = [torch.empty(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(exits, ex, group=group)
        changed = 0
        if rank > 0:
            want = (int(exits[rank - 1][0]), int(exits[rank - 1][1]))
            if want != entry:
                new, new_exit = walker(want[0], want[1], hi)
                traj, new_exit2, ch = splice(new, traj, new_exit, exit_state)
                entry, exit_state = want, new_exit2
                changed = int(ch) | 1   # walked again: the successors must re-check next round
        flag = torch.tensor([changed], dtype=torch.int64)
        dist.all_reduce(flag, group=group)
        if int(flag.item()) == 0:
            break
    # gather the trajectories to rank 0 (a gatherv of int32 triples)
    flat = torch.tensor([v for m in traj for v in m], dtype=torch.int64)
    got = gather_to_root(flat.view(torch.uint8), flat.numel() * 8, group=group)
    if got is None:
        return None
    out: list = []
    for part in got:
        a = part.view(torch.int64).tolist() if part.numel() else []
        out.extend(tuple(a[i:i + 3]) for i in range(0, len(a), 3))
    return out
