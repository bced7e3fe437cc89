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
