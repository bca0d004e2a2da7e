"""Row-split SpMM across the GPUs of a node: one process per GPU, RCCL all-gather of B.

SBP view (oneflow/user/ops/spmm_op.cpp GetSbp): the CSR rows are split by
BalancedSplitter (oneflow/core/common/balanced_splitter.cpp:20-40, the rows OneFlow's S(0) gives,
oneflow/core/job/nd_sbp_util.cpp:68-78), `b` arrives Split(0) and is boxed to Broadcast by an
all-gather (ccl-s-to-b, oneflow/core/boxing/ccl_boxing_function.cpp:185-215 -> ncclAllGather,
oneflow/user/kernels/collective_communication/cuda/cuda_all_gather.cpp:38), `out` is Split(0).

Layout choices (MI355X-first):
  * ncclAllGather needs equal counts, and OneFlow's S->B check wants K % G == 0
    (ccl_boxing_function.cpp:114).  Shards are therefore padded to P = ceil(K/G) rows in the
    gathered buffer, and the local column indices are remapped ONCE at setup (the graph is static
    across layers/iterations) so the hot path needs no compaction copy.
  * The gather is in place: each rank writes its B shard straight into its slot of the gathered
    buffer (`shard_view()`), so no send-buffer copy either.
  * Communication backend: native RCCL through the C-ABI (ofx_comm_*/ofx_allgather) on GPUs;
    torch.distributed (gloo) on CPU for the multi-process CPU tests.
"""
from __future__ import annotations

import ctypes
import datetime
import math
import os
import time

import torch
import torch.distributed as dist

from . import ops
from ._C import balanced_range, current_stream_handle, dtype_code
from ._lib import LIB, PEER_HANDLE_BYTES, PEER_MAX_RANKS, UNIQUE_ID_BYTES, check


def padded_owner_remap(col_idx: torch.Tensor, k: int, world: int) -> torch.Tensor:
    """Column index c of B -> its row in the padded gathered buffer [world * P, n].
    Rank r owns BalancedSplitter(k, world).At(r) and lands at rows [r*P, r*P + size_r)."""
    base, extra = divmod(k, world)
    if extra == 0:
        return col_idx
    c = col_idx.to(torch.int64)
    big = extra * (base + 1)
    owner = torch.where(c < big, c // (base + 1), extra + (c - big) // max(base, 1))
    shift = torch.clamp(owner - extra, min=0)
    return (c + shift).to(col_idx.dtype)


def _exchange_lists(send: list, group, device) -> list:
    """Setup-time all-to-all of variable-length int64 lists (send[p] goes to rank p, result[p]
    came from p) built from all_gather alone — the most portable collective across gloo and
    RCCL; the lists are padded to the longest rank's total for the exchange."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
        else torch.device("cpu")
    counts = torch.tensor([t.numel() for t in send], dtype=torch.int64, device=dev)
    allc = [torch.zeros(world, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allc, counts, group=group)
    cmat = torch.stack(allc).cpu()  # cmat[src, dst] = length of src's list for dst
    width = int(cmat.sum(1).max())
    mine = torch.zeros(max(width, 1), dtype=torch.int64, device=dev)
    flat = torch.cat([t.to(dev, torch.int64) for t in send]) if width else mine[:0]
    mine[: flat.numel()] = flat
    every = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(every, mine, group=group)
    out = []
    for src in range(world):
        off = int(cmat[src, :rank].sum())
        out.append(every[src][off: off + int(cmat[src, rank])].to(device))
    return out


class HaloPlan:
    """Halo-only exchange of B, built once per graph from this rank's
    column indices: each rank receives only the B rows its rows reference, from their owners
    (BalancedSplitter(K, G) shards), and sends the rows its peers asked for.

    Compact B layout on this rank: [own shard rows (K_r) | rows from peer p, p ascending, each
    block in ascending global row order].  `cols` = the column indices remapped into it.  The
    SpMM reads B rows from wherever they live, so the result bits are those of the all-gather.
    """

    def __init__(self, col_idx: torch.Tensor, k: int, world: int, rank: int, group, device):
        lo, hi = balanced_range(k, world, rank)
        self.k_own = hi - lo
        starts = torch.tensor([balanced_range(k, world, r)[0] for r in range(world)],
                              dtype=torch.int64, device=col_idx.device)
        c = col_idx.to(torch.int64)
        uniq = torch.unique(c)  # sorted
        owner = torch.searchsorted(starts, uniq, right=True) - 1
        counts = torch.bincount(owner, minlength=world).cpu()
        first = torch.zeros(world + 1, dtype=torch.int64)
        first[1:] = torch.cumsum(counts, 0)
        need = [uniq[first[p]:first[p + 1]] for p in range(world)]
        need[rank] = need[rank][:0]
        self.recv_counts = [int(counts[p]) if p != rank else 0 for p in range(world)]
        roff, acc = [0] * world, 0
        for p in range(world):
            roff[p] = acc
            acc += self.recv_counts[p]
        self.recv_offsets, self.halo_rows = roff, acc
        self.k_compact = self.k_own + acc
        # remap every nonzero: own -> c - lo; remote from p -> K_r + roff[p] + rank within need[p]
        pos = torch.searchsorted(uniq, c)
        own_ = torch.searchsorted(starts, c, right=True) - 1
        base = torch.tensor([self.k_own + roff[p] - int(first[p]) for p in range(world)],
                            dtype=torch.int64, device=c.device)
        remote = base[own_] + pos
        self.cols = torch.where(own_ == rank, c - lo, remote).to(col_idx.dtype)
        # what my peers need from me: their lists, as rows of my shard
        asked = _exchange_lists(need, group, device)
        self.send_counts = [int(t.numel()) if p != rank else 0 for p, t in enumerate(asked)]
        soff, acc = [0] * world, 0
        for p in range(world):
            soff[p] = acc
            acc += self.send_counts[p]
        self.send_offsets, self.send_rows = soff, acc
        parts = [asked[p] - lo for p in range(world) if p != rank and asked[p].numel()]
        self.send_idx = (torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64)).to(device)
        as_c = lambda v: (ctypes.c_int64 * world)(*v)  # noqa: E731
        self._c = (as_c(self.send_counts), as_c(self.send_offsets), as_c(self.recv_counts),
                   as_c(self.recv_offsets))
        self.remote_rows_total = k - self.k_own


def _copy_rows(dst: torch.Tensor, src: torch.Tensor):
    """dst[i, :] = src[i, :] for two 2-D row-strided views of one shape (HIP on the device)."""
    rows, w = src.shape
    if rows == 0 or w == 0:
        return
    if dst.device.type != "cuda":
        dst.copy_(src)
        return
    esz = src.element_size()
    check(LIB.ofx_gather_rows(current_stream_handle(dst), dtype_code(torch.int64), rows, w * esz,
                              None, src.data_ptr(), src.stride(0) * esz, dst.data_ptr(),
                              dst.stride(0) * esz), "copy_rows")


def _host_staged(group, *tensors) -> bool:
    """gloo moves host memory: device buffers on a gloo group go through host copies (the
    multi-rank GPU tests run several ranks on one GPU, where RCCL refuses the layout)."""
    return dist.get_backend(group) != "nccl" and any(t.is_cuda for t in tensors)


class ExchangeTimeout(RuntimeError):
    """An exchange of B that did not complete within its deadline: a peer that
    never joined.  On the RCCL path the native communicator was aborted first (its queued
    kernels dropped, the peers' calls fail); the message names the exchange."""


def _await(works, deadline_s: float, what: str):
    """Waits for torch.distributed work handles; with deadline_s > 0 a stalled one raises
    ExchangeTimeout instead of blocking forever (the torch/gloo form of ofx_comm_set_timeouts'
    device deadline)."""
    if deadline_s <= 0:
        for w in works:
            w.wait()
        return
    # Work.wait(timeout), not a poll of is_completed(): gloo's point-to-point works only record
    # their completion inside wait(), so a poll never sees them finish
    t0 = time.monotonic()
    for w in works:
        left = max(deadline_s - (time.monotonic() - t0), 1e-3)
        try:
            done = w.wait(timeout=datetime.timedelta(seconds=left))
        except RuntimeError as e:
            raise ExchangeTimeout(f"{what}: not complete after {deadline_s:.1f} s (a peer did not "
                                  f"join the exchange): {e}") from e
        if done is False:
            raise ExchangeTimeout(f"{what}: not complete after {deadline_s:.1f} s "
                                  f"(a peer did not join the exchange)")


def _torch_exchange(send, send_counts, send_offsets, recv, recv_counts, recv_offsets, group,
                    deadline_s: float = 0.0):
    """Grouped point-to-point rows exchange through torch.distributed (the CPU/gloo path of
    ofx_exchange_rows; same counts/offsets convention, rows of the buffers' width)."""
    if _host_staged(group, send, recv):
        host = recv.cpu()
        _torch_exchange(send.cpu(), send_counts, send_offsets, host, recv_counts, recv_offsets,
                        group, deadline_s)
        recv.copy_(host)
        return
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    reqs = []
    for p in range(world):
        if p == rank:
            continue
        gp = dist.get_global_rank(group, p) if group else p
        if send_counts[p]:
            o = send_offsets[p]
            reqs.append(dist.P2POp(dist.isend, send[o:o + send_counts[p]], gp, group))
        if recv_counts[p]:
            o = recv_offsets[p]
            reqs.append(dist.P2POp(dist.irecv, recv[o:o + recv_counts[p]], gp, group))
    if reqs:
        _await(dist.batch_isend_irecv(reqs), deadline_s, "rows exchange")


class GridPlan:
    """The S(0) -> S(0) step on a 2-D grid of the G ranks: R row groups x C column blocks (R*C = G,
    C | N).  Rank p sits in row group g = p // C at column c = p % C; its row group holds the rows
    of ranks g*C .. g*C+C-1 (a contiguous range of OneFlow's S(0) split).

      1. B from row shards to column blocks: every rank sends block c(p) = p % C of its shard to
         each peer p and receives every rank's rows of B[:, its block] (|B|(G-1)/(G*C) per rank;
         the all-gather moves |B|(G-1)/G, the pure column split (C = G) |B|(G-1)/G^2);
      2. SpMM of the row group's rows of A against the N/C columns (the op's S(1) signature
         inside the group; global-form launch on the whole CSR, no slice copy);
      3. C back inside the row group: each member gets its own rows of every block.

    C = 1 is the all-gather itself; C = G is the column split of SURVEY.md §8e alternative (ii)
    ("nsplit").  In between, traffic falls by C while the SpMM's row width shrinks only to N/C
    (the gather runs 512-B rows at 7.7 TB/s but 64-B rows at ~3.9), so the best grid depends on
    the links and N: `tune()` measures every one.

    sub = S > 1 pipelines the step over S column sub-blocks of N/(C*S): the B exchange of
    sub-block s+1 and the C return of sub-block s-1 run on the side stream while the SpMM of
    sub-block s runs (the all-gather's column-block pipelining).  Buffers are
    sub-block-major so every exchange is contiguous per peer:
      send_b [S][C][k_r][w]   (w = N/(C*S); block b, sub-block s = columns b*N/C + s*w ..)
      b_cols [S][K][w]        c_grp [S][group rows][w]        recv_c [S][C][m_r][w]
    Every output column is summed in the same order with the full-width hub schedule
    (split = default_split(N)), so the bits are the row split's for every (C, S)."""

    def __init__(self, owner, cn, row_ptr, col_idx, values, sub: int = 1):
        o = owner
        G, r = o.world, o.rank
        if cn < 1 or G % cn or sub < 1 or o.n % (cn * sub):
            raise ValueError(f"GridPlan: {cn} column blocks must divide world {G}, and {cn} x {sub} "
                             f"sub-blocks n {o.n}")
        self.cn, self.rg, self.sub = cn, G // cn, sub
        self.g, self.c = divmod(r, cn)
        self.ng = o.n // cn
        self.w = w = self.ng // sub
        self.k_rng = [balanced_range(o.k, G, p) for p in range(G)]
        self.m_rng = [balanced_range(o.m, G, p) for p in range(G)]
        members = range(self.g * cn, self.g * cn + cn)
        self.glo, self.ghi = self.m_rng[members[0]][0], self.m_rng[members[-1]][1]
        k_r = self.k_rng[r][1] - self.k_rng[r][0]
        m_r = self.m_rng[r][1] - self.m_rng[r][0]
        self.k_r, self.m_r = k_r, m_r
        m_g = self.ghi - self.glo
        dev, dt = o.device, o.dtype
        self.shard = torch.zeros((k_r, o.n), dtype=dt, device=dev)
        self.send_b = torch.empty((sub, cn, k_r, w), dtype=dt, device=dev)
        self.b_cols = torch.zeros((sub, o.k, w), dtype=dt, device=dev)
        self.c_grp = torch.empty((sub, m_g, w), dtype=dt, device=dev)
        self.recv_c = torch.empty((sub, cn, m_r, w), dtype=dt, device=dev)
        self.csr = (row_ptr, col_idx, values)
        self.nnz_group = int(row_ptr[self.ghi]) - int(row_ptr[self.glo])  # the model's SpMM bytes
        peer = [p != r for p in range(G)]
        mate = [p != r and p // cn == self.g for p in range(G)]
        m_of = lambda p: self.m_rng[p][1] - self.m_rng[p][0]  # noqa: E731
        # per sub-block: (send counts, send offsets, recv counts, recv offsets) in rows of w
        # elements, offsets from the start of the buffer (sub-block s adds s * its stride)
        self.b_counts, self.c_counts = [], []
        for s in range(sub):
            self.b_counts.append((
                [k_r if peer[p] else 0 for p in range(G)],
                [(s * cn + p % cn) * k_r if peer[p] else 0 for p in range(G)],
                [self.k_rng[p][1] - self.k_rng[p][0] if peer[p] else 0 for p in range(G)],
                [s * o.k + self.k_rng[p][0] if peer[p] else 0 for p in range(G)]))
            self.c_counts.append((
                [m_of(p) if mate[p] else 0 for p in range(G)],
                [s * m_g + self.m_rng[p][0] - self.glo if mate[p] else 0 for p in range(G)],
                [m_r if mate[p] else 0 for p in range(G)],
                [(s * cn + p % cn) * m_r if mate[p] else 0 for p in range(G)]))
        as_c = lambda v: (ctypes.c_int64 * G)(*v)  # noqa: E731
        self._cb = [tuple(as_c(v) for v in t) for t in self.b_counts]
        self._cc = [tuple(as_c(v) for v in t) for t in self.c_counts]
        # blocks some peer needs: all of them once there are other row groups
        self.packed = [b for b in range(cn) if b != self.c or self.rg > 1]
        self.kernel = None
        self.events = None
        if dev.type == "cuda":
            # the row group's own nonzeros pick its kernel form (not its share of nnz)
            self.grp_nnz = int(row_ptr[self.ghi]) - int(row_ptr[self.glo])
            self.kernel = ops.SpmmCsrKernel(o.m, o.k, w, col_idx.numel(), o.idx_dtype, dt,
                                            dev, o.options).plan(row_ptr, self.glo, self.ghi,
                                                                 range_nnz=self.grp_nnz)
            self.events = ([torch.cuda.Event() for _ in range(sub)],
                           [torch.cuda.Event() for _ in range(sub)])

    @property
    def name(self) -> str:
        base = "nsplit" if self.rg == 1 else f"grid{self.rg}x{self.cn}"
        return base if self.sub == 1 else f"{base}/s{self.sub}"

    def exchange_rows(self) -> tuple:
        """Elements this rank receives per step: (of B, of C)."""
        return (sum(sum(t[2]) for t in self.b_counts) * self.w,
                sum(sum(t[2]) for t in self.c_counts) * self.w)

    def _cols(self, b, s):
        lo = b * self.ng + s * self.w
        return slice(lo, lo + self.w)

    def _exchange(self, owner, send, counts, c_counts, recv, stream=None):
        if owner.comm_kind == "torch":
            _torch_exchange(send.view(-1, self.w), counts[0], counts[1], recv.view(-1, self.w),
                            counts[2], counts[3], owner.group, owner.exchange_deadline_s)
            return
        sc, so, rc, ro = c_counts
        s = stream if stream is not None else current_stream_handle(recv)
        check(LIB.ofx_exchange_rows(s, owner._comm, dtype_code(owner.dtype), self.w,
                                    send.data_ptr(), sc, so, recv.data_ptr(), rc, ro),
              "exchange_rows")

    def _pack(self, owner):
        lo, hi = self.k_rng[owner.rank]
        if self.shard.device.type == "cuda":
            # two launches: every (sub-block, block) of the shard into send_b, this rank's own
            # block into its rows of b_cols (ofx_copy_blocks, strides in bytes)
            e, w, nb, S, C = self.shard.element_size(), self.w, self.ng, self.sub, self.cn
            k_r, st = self.k_r, current_stream_handle(self.shard)
            if k_r:
                sh, sb, bc = self.shard.data_ptr(), self.send_b.data_ptr(), self.b_cols.data_ptr()
                # blocks some peer needs: all of them with other row groups, else all but c
                ranges = [(0, C)] if self.rg > 1 else [(0, self.c), (self.c + 1, C)]
                for b0, b1 in ranges:
                    if b1 > b0:
                        check(LIB.ofx_copy_blocks(st, S, b1 - b0, k_r, w * e, sh + b0 * nb * e,
                                                  w * e, nb * e, self.shard.stride(0) * e,
                                                  sb + b0 * k_r * w * e, C * k_r * w * e,
                                                  k_r * w * e, w * e), "copy_blocks")
                check(LIB.ofx_copy_blocks(st, S, 1, k_r, w * e, sh + self.c * nb * e, w * e, 0,
                                          self.shard.stride(0) * e, bc + lo * w * e,
                                          owner.k * w * e, 0, w * e), "copy_blocks")
            return
        for s in range(self.sub):
            for b in self.packed:
                _copy_rows(self.send_b[s, b], self.shard[:, self._cols(b, s)])
            _copy_rows(self.b_cols[s, lo:hi], self.shard[:, self._cols(self.c, s)])

    def _spmm(self, owner, s):
        rp, ci, v = self.csr
        if self.kernel is not None:
            self.kernel(rp, ci, v, self.b_cols[s], self.c_grp[s], self.glo, self.ghi, planned=True,
                        range_nnz=self.grp_nnz)
        else:
            ops.spmm_csr_cpu(rp, ci, v, self.b_cols[s], owner.m, owner.k, out=self.c_grp[s],
                             row_begin=self.glo, row_end=self.ghi, options=owner.options)

    def _unpack(self, owner, out):
        lo, hi = self.m_rng[owner.rank]
        if out.device.type == "cuda":
            # the received (sub-block, block)s into out's columns (at most two launches around
            # block c), then this rank's own block from c_grp
            e, w, nb, S, C, m_r = out.element_size(), self.w, self.ng, self.sub, self.cn, self.m_r
            st = current_stream_handle(out)
            if m_r:
                ld = out.stride(0) * e
                rc_, o_ = self.recv_c.data_ptr(), out.data_ptr()
                for b0, b1 in ((0, self.c), (self.c + 1, C)):  # the received blocks
                    if b1 > b0:
                        check(LIB.ofx_copy_blocks(st, S, b1 - b0, m_r, w * e,
                                                  rc_ + b0 * m_r * w * e, C * m_r * w * e,
                                                  m_r * w * e, w * e, o_ + b0 * nb * e, w * e,
                                                  nb * e, ld), "copy_blocks")
                m_g = self.ghi - self.glo
                check(LIB.ofx_copy_blocks(st, S, 1, m_r, w * e,
                                          self.c_grp.data_ptr() + (lo - self.glo) * w * e,
                                          m_g * w * e, 0, w * e,
                                          out.data_ptr() + self.c * nb * e, w * e, 0, ld),
                      "copy_blocks")
            return
        for s in range(self.sub):
            for b in range(self.cn):
                src = (self.c_grp[s, lo - self.glo:hi - self.glo] if b == self.c
                       else self.recv_c[s, b])
                _copy_rows(out[:, self._cols(b, s)], src)

    def exchange_b(self, owner):
        """Phase 1 alone, every sub-block, on the current stream (phase timing)."""
        self._pack(owner)
        for s in range(self.sub):
            self._exchange(owner, self.send_b, self.b_counts[s], self._cb[s], self.b_cols)

    def compute_and_return(self, owner, out):
        """Phases 2 and 3 on the current stream, B exchanged (phase timing)."""
        for s in range(self.sub):
            self._spmm(owner, s)
            if self.cn > 1:
                self._exchange(owner, self.c_grp, self.c_counts[s], self._cc[s], self.recv_c)
        self._unpack(owner, out)
        return out

    def step(self, owner, out):
        """The whole step; with sub-blocks on a GPU, exchanges on the side stream overlap the
        SpMMs (HIP events order them)."""
        if self.sub == 1 or self.kernel is None or owner.comm_kind == "torch":
            self.exchange_b(owner)
            return self.compute_and_return(owner, out)
        cur = torch.cuda.current_stream(owner.device)
        cs = owner.comm_stream
        side = ctypes.c_void_p(cs.cuda_stream)
        ev_b, ev_c = self.events
        self._pack(owner)
        cs.wait_stream(cur)  # packed shard; the previous step's reads of c_grp/recv_c are done
        for s in range(self.sub):
            self._exchange(owner, self.send_b, self.b_counts[s], self._cb[s], self.b_cols, side)
            ev_b[s].record(cs)
        for s in range(self.sub):
            cur.wait_event(ev_b[s])
            self._spmm(owner, s)
            if self.cn > 1:
                ev_c[s].record(cur)
                cs.wait_event(ev_c[s])
                self._exchange(owner, self.c_grp, self.c_counts[s], self._cc[s], self.recv_c, side)
        cur.wait_stream(cs)
        self._unpack(owner, out)
        for t in (self.send_b, self.b_cols, self.c_grp, self.recv_c):
            t.record_stream(cs)
        return out


NSplitPlan = GridPlan  # the C = G grid (kept name: SURVEY.md §8e alternative (ii))


class RowSplitSpmm:
    """out[rows of this rank] = A[rows of this rank, :] @ all_gather(b shards).

    Call with this rank's *local* CSR slice (row_ptr rebased to 0, columns already remapped with
    `remap_columns`) — or construct with `local_csr=False` and pass the full CSR (Broadcast SBP);
    the kernel then computes the row range itself (the OpKernelCache path).

    pipeline = C > 1 splits the dense columns into C blocks of N/C: the gathered buffer is laid
    out block-major [C, K_pad, N/C], block c+1 is all-gathered on a side stream while the SpMM of
    block c runs (out[:, block c] written through ldc = N).  Output columns are independent and
    every block runs the full-N hub schedule (split = default_split(N)), so the result is
    bit-identical to C = 1."""

    def __init__(self, m: int, k: int, n: int, nnz_local: int, dtype: torch.dtype,
                 idx_dtype: torch.dtype, device: torch.device, group=None,
                 comm: str = "auto", local_csr: bool = True, pipeline: int = 1):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.m, self.k, self.n = m, k, n
        self.dtype, self.device = dtype, torch.device(device)
        self.idx_dtype, self.nnz_local = idx_dtype, nnz_local
        self.row_range = balanced_range(m, self.world, self.rank)
        self.k_range = balanced_range(k, self.world, self.rank)
        self.pad = math.ceil(k / self.world) if k else 0
        self.k_padded = self.pad * self.world
        self.local_csr = local_csr
        # every block keeps the hub schedule of the full width (bit-identity across pipelines)
        self.options = ops.make_options(split=ops.default_split(n))
        if comm == "auto":
            comm = "rccl" if self.device.type == "cuda" else "torch"
        if comm not in ("rccl", "rccl-p2p", "rccl-pull", "torch"):
            raise ValueError(f"RowSplitSpmm: unknown comm {comm!r}")
        self.comm_kind = comm
        self._comm = None
        self._peers = None  # (gathered tensor, [peer p's gathered buffer, mapped]) of rccl-pull
        self.comm_stream = None
        if self.device.type == "cuda":
            # high priority: the exchange kernels of a pipelined step get CUs as soon as SpMM
            # workgroups retire instead of queueing behind the whole SpMM grid
            self.comm_stream = torch.cuda.Stream(self.device, priority=-1)
        self.gathered = None
        self.halo = None
        self.ns = None      # the column split (C = G grid), when bound
        self.grids = {}     # name -> GridPlan (every R x C grid with C > 1), when bound
        self.exchange = "allgather"
        self._bound = None
        self.kernel = None
        self.set_pipeline(pipeline)
        if comm.startswith("rccl"):
            self._init_rccl()

    # -- layout ----------------------------------------------------------------------------------
    def set_pipeline(self, chunks: int):
        """(Re)lay out the gathered buffer for `chunks` column blocks, keeping this rank's shard."""
        if chunks < 1 or self.n % chunks:
            raise ValueError(f"RowSplitSpmm: pipeline {chunks} must divide n={self.n}")
        shard = self.shard() if self.gathered is not None else None
        self.gathered = None
        self.chunks, self.nc = chunks, self.n // chunks
        self.gathered = torch.zeros((chunks, self.k_padded, self.nc), dtype=self.dtype,
                                    device=self.device)
        self.chunk_events = ([torch.cuda.Event() for _ in range(chunks)]
                             if self.device.type == "cuda" else None)
        rows_local = self.row_range[1] - self.row_range[0]
        m_kernel = rows_local if self.local_csr else self.m
        self.kernel = None
        if self.device.type == "cuda":
            self.kernel = ops.SpmmCsrKernel(m_kernel, self.k_padded, self.nc, self.nnz_local,
                                            self.idx_dtype, self.dtype, self.device, self.options)
            if self._bound is not None:
                self.kernel.plan(self._bound[0], *self._rows(), range_nnz=self._range_nnz())
        if shard is not None:
            self.load_shard(shard)

    def _rows(self):
        """The kernel's row range: local rows of a local CSR, or this rank's rows of the full one."""
        lo, hi = self.row_range
        return (0, hi - lo) if self.local_csr else (lo, hi)

    def _range_nnz(self) -> int:
        """This rank's nonzeros when its rows are a range of the full CSR (the launch's form
        choice; a local CSR's launch covers all of it, so the count is exact there already)."""
        return 0 if self.local_csr else int(self.nnz_local)

    def _planned(self, row_ptr) -> bool:
        """Launches over the bound CSR reuse the plan built at bind()."""
        return self._bound is not None and row_ptr is self._bound[0]

    def block(self, c: int) -> torch.Tensor:
        """Gathered B, column block c: [K_pad, N/C] contiguous."""
        return self.gathered[c]

    def shard_view(self) -> torch.Tensor:
        """This rank's B shard inside the gathered buffer (write b here: in-place all-gather).
        Only for pipeline 1, where the buffer is plain [K_pad, N]; use load_shard otherwise."""
        if self.chunks != 1:
            raise RuntimeError("shard_view: the gathered buffer is block-major; use load_shard")
        lo, hi = self.k_range
        return self.gathered[0][self.rank * self.pad: self.rank * self.pad + (hi - lo)]

    def load_shard(self, b_shard: torch.Tensor):
        """Writes this rank's rows of B ([K_r, N]) into its slot of every column block."""
        lo, hi = self.k_range
        r0 = self.rank * self.pad
        if b_shard.is_cuda and b_shard.dtype == self.dtype and hi > lo and b_shard.stride(-1) == 1:
            # every column block's slot in one launch
            e = b_shard.element_size()
            check(LIB.ofx_copy_blocks(current_stream_handle(self.gathered), 1, self.chunks, hi - lo,
                                      self.nc * e, b_shard.data_ptr(), 0, self.nc * e,
                                      b_shard.stride(0) * e, self.gathered[0, r0].data_ptr(), 0,
                                      self.k_padded * self.nc * e, self.nc * e), "copy_blocks")
        else:
            for c in range(self.chunks):
                self.gathered[c, r0:r0 + (hi - lo)].copy_(b_shard[:, c * self.nc:(c + 1) * self.nc])
        if self.halo is not None:
            self._load_halo_shard(b_shard)
        for gp in self.grids.values():
            gp.shard.copy_(b_shard)

    def shard(self) -> torch.Tensor:
        lo, hi = self.k_range
        r0 = self.rank * self.pad
        return torch.cat([self.gathered[c, r0:r0 + (hi - lo)] for c in range(self.chunks)], dim=1)

    def remap_columns(self, col_idx: torch.Tensor) -> torch.Tensor:
        """Global B row ids -> rows of the padded gathered buffer (HIP kernel on the device)."""
        if col_idx.device.type != "cuda":
            return padded_owner_remap(col_idx, self.k, self.world)
        col_idx = col_idx.contiguous()
        out = torch.empty_like(col_idx)
        check(LIB.ofx_padded_owner_remap(current_stream_handle(col_idx), dtype_code(col_idx.dtype),
                                         col_idx.numel(), self.k, self.world,
                                         col_idx.data_ptr() if col_idx.numel() else None,
                                         out.data_ptr() if col_idx.numel() else None),
              "padded_owner_remap")
        return out

    # -- communicator (EagerNcclCommMgr::CreateNcclComm pattern: rank 0 makes the id) --------
    def _init_rccl(self):
        uid = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        if self.rank == 0:
            check(LIB.ofx_comm_get_unique_id(uid), "comm_get_unique_id")
        obj = [bytes(uid.raw) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=self.group)
        uid = ctypes.create_string_buffer(obj[0], UNIQUE_ID_BYTES)
        comm = ctypes.c_void_p()
        check(LIB.ofx_set_device(self.device.index if self.device.index is not None else 0), "set_device")
        # bounded: a peer that never joins ends this rank with a named error (and an aborted
        # communicator) instead of a hang inside the set-up; OFX_COMM_TIMEOUT seconds, 300 default
        check(LIB.ofx_comm_init_rank_deadline(ctypes.byref(comm), self.world, uid, self.rank,
                                              self.comm_timeout_s), "comm_init_rank_deadline")
        self._comm = comm
        if self.exchange_deadline_s > 0:
            check(LIB.ofx_comm_set_timeouts(comm, 0.0, self.exchange_deadline_s),
                  "comm_set_timeouts")

    comm_timeout_s = float(os.environ.get("OFX_COMM_TIMEOUT", "300"))
    # seconds an exchange may take to complete, awaited after each one (0 = asynchronous, as in a
    # timed step); OFX_EXCHANGE_DEADLINE sets the default
    exchange_deadline_s = float(os.environ.get("OFX_EXCHANGE_DEADLINE", "0"))

    def set_exchange_deadline(self, seconds: float):
        """Every exchange of this operator (all-gathers, halo and grid send/recv groups) waits for
        its completion for at most `seconds`, then raises ExchangeTimeout naming it -- on RCCL
        after aborting this operator's communicator (ofx_comm_set_timeouts' device deadline, the
        communicator's own).  0 turns the wait off (exchanges stay asynchronous)."""
        self.exchange_deadline_s = float(seconds)
        if self._comm is not None:
            check(LIB.ofx_comm_set_timeouts(self._comm, 0.0, self.exchange_deadline_s),
                  "comm_set_timeouts")

    def abort(self):
        """ncclCommAbort of the native communicator (a stalled rank's watchdog, before it exits):
        peers blocked on this rank then fail instead of waiting forever."""
        if self._comm is not None:
            LIB.ofx_comm_abort(self._comm)  # the handle stays valid: close() frees it

    def comm_size(self):
        """(ranks, this rank) of the native RCCL communicator, None without one."""
        if self._comm is None:
            return None
        nr, rk = ctypes.c_int(), ctypes.c_int()
        check(LIB.ofx_comm_count(self._comm, ctypes.byref(nr), ctypes.byref(rk)), "comm_count")
        return nr.value, rk.value

    def _close_peers(self):
        if self._peers is not None:
            _, ptrs = self._peers
            self._peers = None
            for r, p in enumerate(ptrs):
                if r != self.rank:
                    check(LIB.ofx_peer_close(ctypes.c_void_p(p)), "peer_close")

    def _peer_map(self) -> list:
        """rccl-pull: every rank's gathered buffer, mapped into this process (IPC handles swapped
        over the group once per buffer: after set_pipeline re-lays it out, at the next exchange).
        Collective: every rank reaches it in the same exchange."""
        if self._peers is not None and self._peers[0] is self.gathered:
            return self._peers[1]
        self._close_peers()
        if self.world > PEER_MAX_RANKS:
            raise ValueError(f"rccl-pull: at most {PEER_MAX_RANKS} ranks, not {self.world}")
        h = ctypes.create_string_buffer(PEER_HANDLE_BYTES)
        rc = LIB.ofx_peer_export(ctypes.c_void_p(self.gathered.data_ptr()), h)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(h.raw) if rc == 0 else None, group=self.group)
        if any(x is None for x in handles):  # every rank raises, none waits in a barrier
            raise RuntimeError(f"rccl-pull: ranks {[r for r, x in enumerate(handles) if x is None]} "
                               f"could not export their buffers (rank {self.rank}: rc {rc})")
        ptrs, err = [], None
        try:
            for r, hb in enumerate(handles):
                if r == self.rank:
                    ptrs.append(self.gathered.data_ptr())
                    continue
                ptr = ctypes.c_void_p()
                check(LIB.ofx_peer_open(ctypes.create_string_buffer(hb, PEER_HANDLE_BYTES),
                                        ctypes.byref(ptr)), "peer_open")
                ptrs.append(ptr.value)
        except Exception as e:  # noqa: BLE001 -- agreed on below
            err = f"rank {self.rank}: {e}"
        # every rank learns whether every rank mapped its peers: a rank that raised alone would
        # leave the others blocked in the pull's barriers
        status = [None] * self.world
        dist.all_gather_object(status, err, group=self.group)
        failed = [s for s in status if s is not None]
        if failed:
            for r, p in enumerate(ptrs):
                if r != self.rank:
                    LIB.ofx_peer_close(ctypes.c_void_p(p))
            raise RuntimeError(f"rccl-pull: peer buffers not mapped: {failed[0]}")
        self._peers = (self.gathered, ptrs)
        return ptrs

    def close(self):
        self._close_peers()
        if self._comm is not None:
            check(LIB.ofx_comm_destroy(self._comm), "comm_destroy")
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- the collective ------------------------------------------------------------------------
    def gather_block(self, c: int, stream=None):
        """All-gather column block c in place (each rank's slot is its send buffer)."""
        blk = self.gathered[c]
        slot = blk[self.rank * self.pad:(self.rank + 1) * self.pad]
        count = self.pad * self.nc
        if self.comm_kind == "torch":
            host = blk.cpu() if _host_staged(self.group, blk) else blk
            parts = list(host.view(self.world, self.pad, self.nc).unbind(0))
            work = dist.all_gather(parts, parts[self.rank].clone(), group=self.group,
                                   async_op=True)  # views: in place
            _await([work], self.exchange_deadline_s, f"all-gather of B, column block {c}")
            if host is not blk:
                blk.copy_(host)
            return
        s = stream if stream is not None else current_stream_handle(blk)
        if self.comm_kind == "rccl":
            check(LIB.ofx_allgather(s, slot.data_ptr(), blk.data_ptr(), count,
                                    dtype_code(self.dtype), self._comm), "allgather")
        elif self.comm_kind == "rccl-pull":
            # every peer's block c at the same offset of its buffer as ours
            off = blk.data_ptr() - self.gathered.data_ptr()
            bufs = (ctypes.c_void_p * self.world)(*[p + off for p in self._peer_map()])
            check(LIB.ofx_allgather_pull(s, self._comm, bufs, blk.data_ptr(), count,
                                         dtype_code(self.dtype)), "allgather_pull")
        else:
            check(LIB.ofx_allgather_p2p(s, blk.data_ptr(), count, dtype_code(self.dtype),
                                        self._comm), "allgather_p2p")

    def all_gather_b(self, b_shard: torch.Tensor | None = None):
        if b_shard is not None:
            self.load_shard(b_shard)
        for c in range(self.chunks):
            self.gather_block(c)

    def compute_block(self, c, row_ptr, col_idx, values, out, stream=None):
        lo, hi = self.row_range
        rb, re = self._rows()
        o = out[:, c * self.nc:(c + 1) * self.nc]
        if self.kernel is not None:
            self.kernel(row_ptr, col_idx, values, self.gathered[c], o, rb, re, stream=stream,
                        planned=self._planned(row_ptr), range_nnz=self._range_nnz())
        else:
            m_kernel = hi - lo if self.local_csr else self.m
            ops.spmm_csr_cpu(row_ptr, col_idx, values, self.gathered[c], m_kernel, self.k_padded,
                             out=o, row_begin=rb, row_end=re, options=self.options)

    def compute(self, row_ptr, col_idx, values, out):
        """The local SpMM over the gathered B (B resident; no communication)."""
        for c in range(self.chunks):
            self.compute_block(c, row_ptr, col_idx, values, out)
        return out

    # -- one step ------------------------------------------------------------------------------
    def __call__(self, row_ptr, col_idx, values, b_shard=None, out=None, events=None):
        """Gather + local SpMM.  events: optional (start, mid, end) torch.cuda.Event; with
        pipeline 1 they bracket the gather and the SpMM, pipelined `mid` marks the last gather."""
        lo, hi = self.row_range
        if out is None:
            out = torch.empty((hi - lo, self.n), dtype=self.dtype, device=self.device)
        if b_shard is not None:
            self.load_shard(b_shard)
        pipelined = self.chunks > 1 and self.comm_stream is not None and self.comm_kind != "torch"
        if (not pipelined and not events and self.chunks == 1 and self.comm_kind == "rccl"
                and self.local_csr and self.kernel is not None):
            # the whole step in one C-ABI call: in-place all-gather + local SpMM
            kern = self.kernel
            blk = self.gathered[0]
            opts = kern.launch_options(row_ptr, 0, hi - lo, self._planned(row_ptr))
            check(LIB.ofx_spmm_rowsplit(current_stream_handle(blk), self._comm, kern.idx_dt,
                                        kern.val_dt, hi - lo, self.k_padded, self.n, kern.nnz,
                                        row_ptr.data_ptr(),
                                        col_idx.data_ptr() if col_idx.numel() else None,
                                        values.data_ptr() if values.numel() else None,
                                        blk.data_ptr(), out.data_ptr(), out.stride(0),
                                        kern.workspace.data_ptr(), kern.ws_bytes,
                                        ctypes.byref(opts) if opts else None),
                  "spmm_rowsplit")
            return out
        if events:
            events[0].record()
        if not pipelined:
            self.all_gather_b()
            if events:
                events[1].record()
            self.compute(row_ptr, col_idx, values, out)
        else:
            cur = torch.cuda.current_stream(self.device)
            cs = self.comm_stream
            cs.wait_stream(cur)  # the previous step's reads of the blocks / shard writes are done
            side = ctypes.c_void_p(cs.cuda_stream)
            for c in range(self.chunks):
                self.gather_block(c, stream=side)
                self.chunk_events[c].record(cs)
            if events:
                events[1].record(cs)
            for c in range(self.chunks):
                cur.wait_event(self.chunk_events[c])
                self.compute_block(c, row_ptr, col_idx, values, out)
            # the caching allocator must not recycle these while the side stream uses them
            self.gathered.record_stream(cs)
        if events:
            events[2].record()
        return out

    # -- bound form: this rank's CSR once, every exchange layout prepared ------------------------
    def bind(self, row_ptr, col_idx, values, halo: bool = True, full_csr=None, grid_subs=(1,)):
        """Binds this rank's CSR (`col_idx` in global B row ids; the local slice, or the full CSR
        when local_csr=False).  Remaps the columns for the all-gather layout and, with halo=True,
        builds the halo plan; with `full_csr=(row_ptr, col_idx, values)` of the WHOLE matrix also
        the grid plans: R x C for every C > 1 dividing G, times every sub-block depth S in
        `grid_subs` with C*S | N (C = G is the column split, "nsplit").  `step()` then runs the
        selected exchange."""
        cols = {"allgather": self.remap_columns(col_idx)}
        self.grids, self.ns = {}, None
        if full_csr is not None:
            shard = self.shard()
            cands = {c for c in range(2, self.world + 1) if self.world % c == 0}
            cands.add(self.world)  # one rank: the 1 x 1 "column split" (tests)
            for cn in sorted(cands):
                for sub in grid_subs:
                    if self.n % (cn * sub) == 0:
                        gp = GridPlan(self, cn, *full_csr, sub=sub)
                        gp.shard.copy_(shard)
                        self.grids[gp.name] = gp
            self.ns = self.grids.get("nsplit")
        if halo:
            if self.local_csr:
                mine = col_idx
            else:
                lo, hi = self.row_range
                j0, j1 = int(row_ptr[lo]), int(row_ptr[hi])
                mine = col_idx[j0:j1]
            self.halo = HaloPlan(mine, self.k, self.world, self.rank, self.group, self.device)
            hc = self.halo.cols
            if not self.local_csr:  # full-length array, entries outside this rank's rows unused
                full = torch.zeros_like(col_idx)
                full[j0:j1] = hc
                hc = full
            cols["halo"] = hc
            self.compact = None
            self.set_halo_pipeline(1, row_ptr=row_ptr, nnz=col_idx.numel())
        self._bound = (row_ptr, cols, values)
        if self.kernel is not None:
            self.kernel.plan(row_ptr, *self._rows(), range_nnz=self._range_nnz())

    def set_halo_pipeline(self, chunks: int, row_ptr=None, nnz=None):
        """(Re)lays out the halo buffers for `chunks` column blocks of N/C, block-major like the
        all-gather's: compact B [C, K_own + halo rows, N/C] and the rows peers asked for
        [C, send rows, N/C], so every block's exchange is one contiguous run per peer.  Block c+1
        is packed and exchanged on the side stream while the SpMM of block c runs; every block
        keeps the full-width hub schedule, so the bits are those of chunks = 1.  Keeps the shard."""
        h = self.halo
        if h is None:
            raise RuntimeError("set_halo_pipeline: bind(halo=True) first")
        if chunks < 1 or self.n % chunks:
            raise ValueError(f"RowSplitSpmm: halo pipeline {chunks} must divide n={self.n}")
        row_ptr = row_ptr if row_ptr is not None else self._bound[0]
        nnz = nnz if nnz is not None else self._bound[1]["halo"].numel()
        shard = self._halo_shard() if self.compact is not None else self.shard()
        nc = self.n // chunks
        self.halo_chunks, self.halo_nc = chunks, nc
        self.compact = torch.zeros((chunks, h.k_compact, nc), dtype=self.dtype, device=self.device)
        self.send_buf = torch.empty((chunks, h.send_rows, nc), dtype=self.dtype, device=self.device)
        self.halo_events = None
        self.halo_kernel = None
        if self.device.type == "cuda":
            self.halo_events = [torch.cuda.Event() for _ in range(chunks)]
            rows_local = self.row_range[1] - self.row_range[0]
            self.halo_kernel = ops.SpmmCsrKernel(rows_local if self.local_csr else self.m,
                                                 h.k_compact, nc, nnz, self.idx_dtype, self.dtype,
                                                 self.device, self.options).plan(
                                                     row_ptr, *self._rows(),
                                                     range_nnz=self._range_nnz())
        self._load_halo_shard(shard)

    def _load_halo_shard(self, b_shard: torch.Tensor):
        k_own, nc = self.halo.k_own, self.halo_nc
        for c in range(self.halo_chunks):
            self.compact[c, :k_own].copy_(b_shard[:, c * nc:(c + 1) * nc])

    def _halo_shard(self) -> torch.Tensor:
        return torch.cat(list(self.compact[:, : self.halo.k_own].unbind(0)), dim=1)

    def _halo_block(self, c: int, stream=None):
        """Block c: pack the rows each peer asked for, then grouped send/recv into compact[c]."""
        h = self.halo
        comp, send = self.compact[c], self.send_buf[c]
        if self.comm_kind == "torch":
            if h.send_rows:
                torch.index_select(comp, 0, h.send_idx, out=send)
            _torch_exchange(send, h.send_counts, h.send_offsets, comp,
                            h.recv_counts, [h.k_own + o for o in h.recv_offsets], self.group,
                            self.exchange_deadline_s)
            return
        s = stream if stream is not None else current_stream_handle(comp)
        esz, nc = comp.element_size(), self.halo_nc
        if h.send_rows:
            check(LIB.ofx_gather_rows(s, dtype_code(torch.int64), h.send_rows, nc * esz,
                                      h.send_idx.data_ptr(), comp.data_ptr(), nc * esz,
                                      send.data_ptr(), nc * esz), "gather_rows")
        sc, so, rc, ro = h._c
        check(LIB.ofx_exchange_rows(s, self._comm, dtype_code(self.dtype), nc,
                                    send.data_ptr() if h.send_rows else None, sc, so,
                                    comp.data_ptr() + h.k_own * nc * esz, rc, ro),
              "exchange_rows")

    def halo_exchange(self, b_shard=None):
        """Every block's pack + exchange on the current stream."""
        if b_shard is not None:
            self._load_halo_shard(b_shard)
        for c in range(self.halo_chunks):
            self._halo_block(c)

    def _halo_compute_block(self, c: int, out):
        row_ptr, cols, values = self._bound
        lo, hi = self.row_range
        rb, re = (0, hi - lo) if self.local_csr else (lo, hi)
        nc = self.halo_nc
        o = out[:, c * nc:(c + 1) * nc]
        if self.halo_kernel is not None:
            self.halo_kernel(row_ptr, cols["halo"], values, self.compact[c], o, rb, re, planned=True,
                             range_nnz=self._range_nnz())
        else:
            m_kernel = hi - lo if self.local_csr else self.m
            ops.spmm_csr_cpu(row_ptr, cols["halo"], values, self.compact[c], m_kernel,
                             self.halo.k_compact, out=o, row_begin=rb, row_end=re,
                             options=self.options)

    def halo_compute(self, out):
        for c in range(self.halo_chunks):
            self._halo_compute_block(c, out)
        return out

    def _halo_step(self, out, b_shard=None, events=None):
        pipelined = (self.halo_chunks > 1 and self.comm_stream is not None
                     and self.comm_kind != "torch" and not events)
        if not pipelined:
            if events:
                events[0].record()
            self.halo_exchange(b_shard)
            if events:
                events[1].record()
            self.halo_compute(out)
            if events:
                events[2].record()
            return out
        if b_shard is not None:
            self._load_halo_shard(b_shard)
        cur = torch.cuda.current_stream(self.device)
        cs = self.comm_stream
        cs.wait_stream(cur)  # shard written; the previous step's reads of the blocks are done
        side = ctypes.c_void_p(cs.cuda_stream)
        for c in range(self.halo_chunks):
            self._halo_block(c, stream=side)
            self.halo_events[c].record(cs)
        for c in range(self.halo_chunks):
            cur.wait_event(self.halo_events[c])
            self._halo_compute_block(c, out)
        cur.wait_stream(cs)
        for t in (self.compact, self.send_buf):
            t.record_stream(cs)
        return out

    def step(self, out, b_shard=None, events=None):
        """One exchange + local SpMM over the bound CSR with the selected exchange."""
        row_ptr, cols, values = self._bound
        if self.exchange in self.grids:
            gp = self.grids[self.exchange]
            if b_shard is not None:
                gp.shard.copy_(b_shard)
            if not events:
                return gp.step(self, out)
            events[0].record()
            gp.exchange_b(self)
            events[1].record()
            gp.compute_and_return(self, out)
            events[2].record()
            return out
        if self.exchange == "halo":
            return self._halo_step(out, b_shard, events)
        if b_shard is not None:
            self.load_shard(b_shard)
        return self(row_ptr, cols["allgather"], values, out=out, events=events)

    def gather_phase(self):
        """The exchange alone (phase timing)."""
        if self.exchange == "halo":
            self.halo_exchange()
        elif self.exchange in self.grids:
            self.grids[self.exchange].exchange_b(self)
        else:
            self.all_gather_b()

    def compute_phase(self, out):
        """The local SpMM alone with the exchanged B resident (phase timing)."""
        if self.exchange == "halo":
            return self.halo_compute(out)
        if self.exchange in self.grids:  # local SpMM + the return of C inside the row group
            return self.grids[self.exchange].compute_and_return(self, out)
        row_ptr, cols, values = self._bound
        return self.compute(row_ptr, cols["allgather"], values, out)

    # -- schedule choice -------------------------------------------------------------------------
    # A-priori model of one step per exchange candidate: bytes this rank receives
    # at R_X plus the local SpMM's gather-model bytes at R_HBM (B rows of fewer than 128 B cost a
    # whole 128-B line, "Narrow rows"); with D pipeline blocks / sub-blocks the two overlap:
    # max(x, s) + min(x, s) / D.  R_X is an xGMI assumption (RCCL reaching 300 GB/s of ingress per
    # GPU over 7 links of ~153 GB/s); `tune` refits it to the first measured candidate before it
    # prunes.
    R_X = 300e9
    R_HBM = 6.0e12

    def _spmm_bytes(self, rows, nnz, w, blocks=1):
        e = torch.empty(0, dtype=self.dtype).element_size()
        return blocks * (4 * (rows + 1) + (4 + e) * nnz + max(e * w, 128) * nnz + e * rows * w)

    def _candidate_model(self, name, chunks):
        """(bytes received per step, local SpMM bytes, overlap depth) of a candidate."""
        e = torch.empty(0, dtype=self.dtype).element_size()
        rows = self.row_range[1] - self.row_range[0]
        if name in self.grids:
            gp = self.grids[name]
            b_el, c_el = gp.exchange_rows()
            return ((b_el + c_el) * e, self._spmm_bytes(gp.ghi - gp.glo, gp.nnz_group, gp.w, gp.sub),
                    gp.sub)
        if name == "halo":
            recv = self.halo.halo_rows * self.n * e
        else:
            recv = (self.k_padded - self.pad) * self.n * e
        return recv, self._spmm_bytes(rows, self.nnz_local, self.n // chunks, chunks), chunks

    @staticmethod
    def _model_ms(recv, spmm, depth, r_x, r_h):
        x, t = recv / r_x * 1e3, spmm / r_h * 1e3
        return x + t if depth <= 1 else max(x, t) + min(x, t) / depth

    # exchange candidates that keep the north star's 1-D row split: every rank
    # owns its BalancedSplitter rows at full width; grids / the column split are 2-D partitions
    @staticmethod
    def is_rowsplit_exchange(name: str) -> bool:
        return not name.startswith(("grid", "nsplit"))

    @classmethod
    def pick_best(cls, times: dict, rowsplit_only: bool):
        """The fastest finite candidate of `times` ({name: ms}); with `rowsplit_only` the fastest
        1-D row-split one (None if none completed).  Ties go to the name first in sort order."""
        pool = {nm: ms for nm, ms in times.items() if math.isfinite(ms)
                and (not rowsplit_only or cls.is_rowsplit_exchange(nm))}
        return min(sorted(pool), key=pool.get) if pool else None

    def describe(self) -> str:
        """The partition and exchange this operator runs, as the bench's config.parallelism
        names it (built from the kept exchange, never a constant)."""
        w = self.world
        if self.exchange in self.grids:
            gp = self.grids[self.exchange]
            return (f"2-D grid {gp.rg}x{gp.cn} over {w} ranks ({self.exchange}): row groups x "
                    f"column blocks, B exchanged by {self.comm_kind} send/recv, C returned in the "
                    f"row group; sub-blocks {gp.sub}")
        via = {"rccl": "RCCL ring all-gather (ncclAllGather)",
               "rccl-p2p": "RCCL grouped send/recv all-gather",
               "rccl-pull": "IPC peer-pull all-gather (RCCL barriers)",
               "torch": "torch.distributed all-gather"}[self.comm_kind]
        if self.exchange == "halo":
            via = {"torch": "torch.distributed"}.get(self.comm_kind, "RCCL") + \
                " grouped send/recv of the halo rows only"
            depth = self.halo_chunks
        else:
            via += " of the padded Split(0) shards of B"
            depth = self.chunks
        overlap = self.comm_stream is not None and self.comm_kind != "torch"
        pipe = (f", {depth} column blocks " + ("pipelined on a side stream" if overlap
                                                else "in sequence")) if depth > 1 else ""
        return f"1-D row split x{w} (BalancedSplitter rows) + {via}{pipe}"

    # tests only: "name-prefix:factor[,...]" multiplies the measured time of matching candidates
    # (a grid made to look fastest, to check the 1-D choice); never set in a measured run
    _TEST_SCALE_ENV = "OFX_TUNE_TEST_SCALE"

    def tune(self, out, pipelines=(1, 2, 4), reps: int = 3, force: bool = False,
             budget_s: float | None = None, prune: float = 3.0,
             first: tuple | None = None, log=None, on_candidate=None,
             rowsplit_only: bool = False, kinds: tuple | None = None) -> dict:
        """Times every exchange on this node with the real step over the bound CSR: all-gather
        (ring / point-to-point) x pipeline depth, the halo exchange and the grid plans if built.
        Keeps the fastest -- with `rowsplit_only`, the fastest 1-D row-split candidate (all-gather
        or halo: the north star's partition); grids are then still measured, after every 1-D
        candidate, and reported in `self.tune_best_2d` but never kept.  Timings are max-reduced
        over ranks, so all ranks choose the same; every candidate produces the same bytes.
        Returns {"<comm>/p<C>" | "halo[/p<C>]" | "nsplit[/s<S>]" | "grid<R>x<C>[/s<S>]": ms} of
        the candidates measured.

        The all-gather kinds are `kinds`, default ring + grouped point-to-point.  The IPC peer
        pull ("rccl-pull") is opt-in (kinds=(..., "rccl-pull") or RowSplitSpmm(comm="rccl-pull")
        pinned by the caller): its cross-GPU visibility has not run on two devices yet.

        Order and bounds (so the first 8-GPU run ends in bounded time): the candidates named in
        `first` (default: the plain row split + all-gather of the north star, "<comm>/p1"; without
        `rowsplit_only` also the 2x4 grid with sub-block overlap), then the rest in ascending
        model time (_model_ms), 1-D candidates before grids under `rowsplit_only`.  After the
        first measurement R_X is refitted to it; a candidate whose refitted model time exceeds
        `prune` x the best measured time is skipped, and once `budget_s` seconds have passed (max
        over ranks) the rest are skipped.  The plain all-gather is never skipped (VERDICT r3 item
        4: the north star's number is always measured, whichever candidate wins).
        `on_candidate(name)` is called before each measurement (the bench's per-rank phase log
        and watchdog).  Each candidate's first (untimed) step runs under the exchange deadline
        (a peer that never joins is named); its timed reps run with the deadline off, as the
        timed steps do, so a pipelined exchange overlaps its SpMM there too.
        Every decision uses max-reduced values, so all ranks take the same path.  The record is in
        `self.tune_report`: per candidate the model time, the measured time and the status.
        One rank has nothing to exchange, so it keeps its setting unless `force` (tests).  With
        torch.distributed as the transport (gloo on CPU, the tests) the all-gather candidates are
        its collectives and the clock is the host's."""
        if self._bound is None:
            raise RuntimeError("tune: bind() the CSR first")
        self.tune_report = {}
        self.tune_best_2d = None
        if self.world == 1 and not force:
            return {}
        native = self.comm_kind.startswith("rccl")
        if kinds is None:
            kinds = ("rccl", "rccl-p2p") if native else ("torch",)
        if native:
            bad = [kd for kd in kinds if kd not in ("rccl", "rccl-p2p", "rccl-pull")]
            if "rccl-pull" in kinds and self.world > PEER_MAX_RANKS:
                bad.append("rccl-pull")
        else:
            bad = [kd for kd in kinds if kd != "torch"]
        if bad:
            raise ValueError(f"tune: all-gather kinds {bad} not available on this communicator")
        test_scale = []
        for item in filter(None, os.environ.get(self._TEST_SCALE_ENV, "").split(",")):
            pre, _, f = item.partition(":")
            test_scale.append((pre, float(f)))
        base = "rccl" if native else "torch"
        on_gpu = self.device.type == "cuda"
        red_dev = self.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")

        def max_over_ranks(v: float) -> float:
            t = torch.tensor([v], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            return float(t.item())

        ref_digest = []

        def digest():
            # every candidate writes the same bytes: a weighted sum of a strided
            # sample of this rank's output bits (<= 4M elements), compared with the first one's
            bits = out.reshape(-1).view({2: torch.int16, 4: torch.int32, 8: torch.int64}[out.element_size()])
            step = max(1, bits.numel() // 4_000_000)
            x = bits[::step].to(torch.int64)
            w = torch.arange(x.numel(), dtype=torch.int64, device=x.device) % 1_000_003 + 1
            return int((x * w).sum().item()), int(x.numel())

        def measure():
            # A candidate that raises on any rank (a host-side error, deterministic across ranks)
            # is timed as +inf everywhere by the max-reduce, so no rank keeps it; so is one whose
            # output differs from the first candidate's on any rank (a wrong exchange).
            ms = float("inf")
            deadline = self.exchange_deadline_s
            try:
                self.step(out)  # untimed, under the deadline: every exchange awaited
                if on_gpu:
                    torch.cuda.synchronize(self.device)
                if deadline > 0:  # the timed reps run as the timed steps do: asynchronous
                    self.set_exchange_deadline(0)
                if on_gpu:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(reps):
                        self.step(out)
                    e1.record()
                    torch.cuda.synchronize(self.device)
                    ms = e0.elapsed_time(e1) / reps
                else:
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        self.step(out)
                    ms = (time.perf_counter() - t0) * 1e3 / reps
            except ExchangeTimeout:
                raise  # a peer that never joined: no candidate can be timed, the rank ends
            except Exception as e:  # noqa: BLE001 -- reported, candidate dropped
                self.tune_errors[f"{self.exchange}/{self.comm_kind}/p{self.chunks}"] = repr(e)
            finally:
                if deadline > 0 and self.exchange_deadline_s != deadline:
                    self.set_exchange_deadline(deadline)
            for pre, f in test_scale:
                if cur_name[0].startswith(pre):
                    ms *= f
            ms = max_over_ranks(ms)
            if not math.isfinite(ms):
                return ms
            d = digest()
            if not ref_digest:  # the first candidate every rank ran: the reference bytes
                ref_digest.append(d)
                return ms
            if max_over_ranks(1.0 if d != ref_digest[0] else 0.0) > 0:
                self.tune_errors[f"{self.exchange}/{self.comm_kind}/p{self.chunks}"] = \
                    "output differs from the first candidate's"
                return float("inf")
            return ms

        # the candidates: (name, setter)
        cands = []
        for chunks in pipelines:
            if self.n % chunks == 0:
                for kind in kinds:
                    def ag(chunks=chunks, kind=kind):
                        self.exchange = "allgather"
                        self.set_pipeline(chunks)
                        self.comm_kind = kind
                    cands.append((f"{kind}/p{chunks}", ag, "allgather", chunks))
        if self.halo is not None:
            for chunks in pipelines:
                if self.n % chunks == 0:
                    def hl(chunks=chunks):
                        self.set_pipeline(1)
                        self.set_halo_pipeline(chunks)
                        self.exchange, self.comm_kind = "halo", base
                    cands.append(("halo" if chunks == 1 else f"halo/p{chunks}", hl, "halo", chunks))
        for name in self.grids:
            def gr(name=name):
                self.set_pipeline(1)
                self.exchange, self.comm_kind = name, base
            cands.append((name, gr, name, 1))
        # the model inputs of every candidate, max-reduced over ranks: the order and every skip
        # decision below are then the same on all ranks (their collectives stay matched)
        model = {c[0]: self._candidate_model(c[2], c[3]) for c in cands}
        names = sorted(model)
        mt = torch.tensor([[model[nm][0], model[nm][1]] for nm in names], dtype=torch.float64,
                          device=red_dev)
        dist.all_reduce(mt, op=dist.ReduceOp.MAX, group=self.group)
        model = {nm: (float(mt[i, 0]), float(mt[i, 1]), model[nm][2]) for i, nm in enumerate(names)}
        prior = {nm: self._model_ms(*model[nm], self.R_X, self.R_HBM) for nm in model}
        always = {f"{base}/p1"}
        if first is None:
            first = (f"{base}/p1",) if rowsplit_only else (f"{base}/p1", "grid2x4/s2")
        oned = self.is_rowsplit_exchange
        cands.sort(key=lambda c: (c[0] not in first,
                                  first.index(c[0]) if c[0] in first else 0,
                                  rowsplit_only and not oned(c[0]), prior[c[0]], c[0]))

        times = {}
        self.tune_errors = {}
        r_x = self.R_X
        t_start = time.perf_counter()
        cur_name = [None]
        for name, setter, _, _ in cands:
            cur_name[0] = name
            rec = {"predicted_ms": round(prior[name], 4), "recv_mb": round(model[name][0] / 1e6, 2),
                   "spmm_mb": round(model[name][1] / 1e6, 2)}
            self.tune_report[name] = rec
            best = min(times.values()) if times else float("inf")
            fitted = self._model_ms(*model[name], r_x, self.R_HBM)
            rec["refit_predicted_ms"] = round(fitted, 4)
            if name not in always:
                if (budget_s is not None and times
                        and max_over_ranks(time.perf_counter() - t_start) > budget_s):
                    rec["status"] = "skipped: budget"
                    continue
                if math.isfinite(best) and fitted > prune * best:
                    rec["status"] = "skipped: model"
                    continue
            if on_candidate is not None:
                on_candidate(name)
            setter()
            ms = measure()
            rec["measured_ms"] = round(ms, 4) if math.isfinite(ms) else None
            rec["status"] = "measured" if math.isfinite(ms) else "error"
            if log is not None:
                log(f"[tune] {name}: {ms:.3f} ms (model {prior[name]:.3f}, refit {fitted:.3f}; "
                    f"{time.perf_counter() - t_start:.1f} s)")
            if math.isfinite(ms):
                times[name] = ms
                if len(times) == 1:  # refit the exchange rate to the first measurement
                    recv, spmm, depth = model[name]
                    t_ms = spmm / self.R_HBM * 1e3
                    if depth <= 1:
                        x_ms = ms - t_ms
                    elif ms - t_ms / depth >= t_ms:  # exchange-bound: ms = x + t / D
                        x_ms = ms - t_ms / depth
                    else:  # SpMM-bound: ms = t + x / D
                        x_ms = depth * (ms - t_ms)
                    if recv > 0 and x_ms > 0:
                        r_x = recv / (x_ms * 1e-3)
        self.tune_rate_fit = r_x
        if not times:
            raise RuntimeError(f"RowSplitSpmm.tune: every exchange failed: {self.tune_errors}")
        best = self.pick_best(times, rowsplit_only)
        two_d = {nm: ms for nm, ms in times.items() if not oned(nm)}
        if two_d:
            g = min(two_d, key=two_d.get)
            self.tune_best_2d = (g, two_d[g])
        if best is None:
            raise RuntimeError(f"RowSplitSpmm.tune: no 1-D row-split exchange completed: "
                               f"{self.tune_errors}")
        if self.halo is not None:
            self.set_halo_pipeline(int(best.split("/p")[1]) if best.startswith("halo/p") else 1)
        if best.startswith("halo"):
            self.exchange, self.comm_kind = "halo", base
            self.set_pipeline(1)
        elif best in self.grids:
            self.exchange, self.comm_kind = best, base
            self.set_pipeline(1)
        else:
            kind, p = best.split("/p")
            self.exchange, self.comm_kind = "allgather", kind
            self.set_pipeline(int(p))
        return times
