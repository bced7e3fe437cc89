"""Chromosome sharding across GPUs and the gather of per-chromosome record streams.

SCCG compresses one chromosome pair per invocation and pairs are independent,
so the multi-GPU job is: LPT-assign pairs to ranks (largest target first onto the least-loaded
rank), compress locally, then move every rank's record texts to rank 0 -- the job's only data
exchange -- with one size all-gather and one padded all-gather (RCCL over xGMI with the "nccl"
backend on GPUs; "gloo" on CPU for tests).
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


def gather_records(parts: dict[str, bytes | torch.Tensor], device: torch.device | None = None,
                   group=None) -> dict[str, bytes] | None:
    """Gather {chromosome: record text} from every rank to rank 0.

    `parts` values may be bytes or uint8 tensors (device tensors stay on the device for RCCL).
    Returns the merged dict on rank 0, None elsewhere."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = device or torch.device("cpu")
    names = sorted(parts)
    blobs = []
    for n in names:
        v = parts[n]
        blobs.append(v.to(dev) if isinstance(v, torch.Tensor) else torch.frombuffer(bytearray(v), dtype=torch.uint8).to(dev)
                     if len(v) else torch.zeros(0, dtype=torch.uint8, device=dev))
    # header: one length per chromosome name and one per blob, both variable -> gather sizes first
    name_bytes = "\0".join(names).encode()
    lens = torch.tensor([len(name_bytes)] + [int(b.numel()) for b in blobs] + [len(blobs)], dtype=torch.int64,
                        device=dev)
    n_lens = torch.tensor([lens.numel()], dtype=torch.int64, device=dev)
    all_n = [torch.zeros_like(n_lens) for _ in range(world)]
    dist.all_gather(all_n, n_lens, group=group)
    maxn = int(max(int(x.item()) for x in all_n))
    padded_lens = torch.zeros(maxn, dtype=torch.int64, device=dev)
    padded_lens[: lens.numel()] = lens
    all_lens = [torch.zeros_like(padded_lens) for _ in range(world)]
    dist.all_gather(all_lens, padded_lens, group=group)
    payload = torch.cat([torch.frombuffer(bytearray(name_bytes), dtype=torch.uint8).to(dev)
                         if name_bytes else torch.zeros(0, dtype=torch.uint8, device=dev)] + blobs)
    sizes = []
    for r in range(world):
        ln = all_lens[r][: int(all_n[r].item())].tolist()
        sizes.append(sum(ln[:-1]))
    mx = max(sizes) if sizes else 0
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    buf[: payload.numel()] = payload
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    if rank != 0:
        return None
    merged: dict[str, bytes] = {}
    for r in range(world):
        ln = all_lens[r][: int(all_n[r].item())].tolist()
        nb, blob_lens = ln[0], ln[1:-1]
        raw = bufs[r].cpu().numpy().tobytes()
        rnames = raw[:nb].decode().split("\0") if nb else []
        off = nb
        for name, L in zip(rnames, blob_lens):
            merged[name] = raw[off: off + L]
            off += L
    return merged
