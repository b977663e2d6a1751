"""Multi-GPU image tiling for the path tracer: one process per GPU (torch.distributed over RCCL/xGMI).

Pixels are independent and the RNG is keyed by the GLOBAL pixel index, so an N-rank render is
bitwise identical to a 1-rank render.  Rows are dealt to ranks in bands of `band` rows round-robin
(band b -> rank b % N), which balances the sky rows at the top/bottom of the frame against the box in
the middle.  The only collective is the final RGBA8 all-gather (the RCCL framebuffer gather of
BASELINE.json's C4/C5 configurations); there is no exchange during rendering.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on device tensors, "gloo" on CPU
tensors (the multi-process CPU tests).
"""
import torch
import torch.distributed as dist


def local_rows(H, band, rank, nranks):
    """Global row indices owned by `rank`, in local order (the C-ABI's local row order)."""
    rows = []
    b = rank
    while b * band < H:
        rows.extend(range(b * band, min((b + 1) * band, H)))
        b += nranks
    return rows


class ImageGather:
    """Preallocated all-gather of per-rank RGBA8 row sets + reassembly on rank 0."""

    def __init__(self, W, H, band, rank, nranks, device, collective=None):
        """collective: run the all-gather even with one rank (bench.py --force-dist: the RCCL path exercised on a
        one-GPU box); default: only when nranks > 1."""
        self.W, self.H, self.rank, self.nranks = W, H, rank, nranks
        self.collective = nranks > 1 if collective is None else bool(collective)
        rows = [local_rows(H, band, r, nranks) for r in range(nranks)]
        self.max_rows = max(len(r) for r in rows)
        self.n_local = len(rows[rank])
        self.send = torch.zeros(self.max_rows * W, dtype=torch.int32, device=device)
        self.recv = torch.zeros(nranks * self.max_rows * W, dtype=torch.int32, device=device) if self.collective else self.send
        self.image = torch.zeros(H * W, dtype=torch.int32, device=device)
        src, dst = [], []
        for r in range(nranks):
            for i, y in enumerate(rows[r]):
                src.append(r * self.max_rows + i)
                dst.append(y)
        self.src = torch.tensor(src, dtype=torch.int64, device=device)
        self.dst = torch.tensor(dst, dtype=torch.int64, device=device)

    def local_view(self):
        """The send buffer's first n_local rows (fill it with this rank's RGBA8 rows)."""
        return self.send[: self.n_local * self.W]

    def gather(self):
        """All-gather the row sets; rank 0 scatters them into image (H*W int32, row 0 = bottom)."""
        if self.collective:
            if self.send.is_cuda:
                dist.all_gather_into_tensor(self.recv, self.send)
            else:   # gloo has no all_gather_into_tensor on every torch build
                parts = list(self.recv.view(self.nranks, -1).unbind(0))   # views into recv
                dist.all_gather(parts, self.send)
        if self.rank == 0:
            self.image.view(self.H, self.W).index_copy_(0, self.dst, self.recv.view(-1, self.W).index_select(0, self.src))
        return self.image
