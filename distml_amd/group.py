"""Multi-GPU shard group: one process per GPU, RCCL over xGMI via torch.distributed.

The matrix's rows are split by KeyRange.linearSplit (KeyRange.java:68-80,
DMatrix.partition DMatrix.java:53-64); rank r owns shard r in HBM.

Path for device-resident FULL-RANGE pushes (every push covers all rows — the
data-parallel gradient case):
  1. pre-reduce: the rank's W local pushes, in push order, into one partial
     buffer of the whole matrix (dml_reduce_buckets_dense, HBM-bound);
  2. reduce-scatter (sum) of the partials: rank r receives the sum of every
     rank's partial for its shard (RCCL ncclReduceScatter over xGMI);
  3. owner apply: shard += received (dml_store_apply_dense_device).
fp32 results differ from the single-shard ordered sum only by summation order
(bound stated in tests/test_group_gloo.py); int32 is exact.

Pushes that are already split per shard (SparseMatrix.push splits by partition,
SparseMatrix.java:46-60) need no exchange: push_local() applies them on the
owner with the exact ordered reduce.

int32 matrices (IntMatrixStore): the owner apply checks the final counters
(IntMatrixStore.java:174-176) and reports the first negative element of the
first failing call (row-major) at the next call or flush(); the store then
refuses later applies. A counter that dips below zero only between two pushes
of one pre-reduced sum is not seen (the reference would throw there) — the
divergence SURVEY.md §8c names for batched reduces. push_exchange() applies
int32 pushes exactly, intermediates included.

Buffer contract of the asynchronous paths (push_full_range, push_exchange,
push_local): the push buffers must stay allocated and unmodified until flush()
— the same contract as dml_store_push_batch_device. The group orders its own
reads after the work the caller's current stream enqueued before the call.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

from . import _lib
from .datadesc import DataDesc, KeyRange
from .store import DataStore, check


class HipOps:
    """Product kernels (libdistml_ps). Tests may inject CPU stand-ins with the same methods."""

    def prereduce(self, fmt: DataDesc, first: int, rows: int, cols: int, dev_ptrs: Sequence[int],
                  lens: Sequence[int], out_ptr: int, stream: int) -> None:
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        rc = _lib.load().dml_reduce_buckets_dense(C.byref(fmt.to_c()), first, rows, cols, ptrs, ls, n,
                                                   C.c_void_p(out_ptr), C.c_void_p(stream))
        check(rc)

    def apply(self, store: DataStore, src_ptr: int, elems: int) -> None:
        check(_lib.load().dml_store_apply_dense_device(store._h, C.c_void_p(src_ptr), elems), store)

    # piecewise pre-reduce (pipelined with the reduce-scatter)
    def begin(self, fmt: DataDesc, first: int, rows: int, cols: int, dev_ptrs, lens, stream: int):
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        h = C.c_void_p()
        check(_lib.load().dml_prereduce_begin(C.byref(fmt.to_c()), first, rows, cols, ptrs, ls, n,
                                              C.c_void_p(stream), C.byref(h)))
        return h.value

    def piece(self, h, block: int, stride: int, off: int, ntask_rows: int, out_ptr: int, stream: int) -> None:
        check(_lib.load().dml_prereduce_piece(C.c_void_p(h), block, stride, off, ntask_rows, C.c_void_p(out_ptr),
                                              C.c_void_p(stream)))

    def end(self, h) -> None:
        check(_lib.load().dml_prereduce_end(C.c_void_p(h)))

    # speculative pre-reduce within a context (dml_prectx_*)
    def ctx_create(self, fmt: DataDesc, first: int, rows: int, cols: int, device: int):
        h = C.c_void_p()
        check(_lib.load().dml_prectx_create(C.byref(fmt.to_c()), first, rows, cols, device, C.byref(h)))
        return h.value

    def ctx_destroy(self, ctx) -> None:
        _lib.load().dml_prectx_destroy(C.c_void_p(ctx))

    def ctx_stats(self, ctx, reset: bool = False) -> dict:
        c = _lib.dml_store_counters()
        check(_lib.load().dml_prectx_stats(C.c_void_p(ctx), C.byref(c), int(reset)))
        return {f: getattr(c, f) for f, _ in c._fields_}

    def begin_ctx(self, ctx, dev_ptrs, lens, stream: int):
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        h = C.c_void_p()
        check(_lib.load().dml_prereduce_begin_ctx(C.c_void_p(ctx), ptrs, ls, n, C.c_void_p(stream), C.byref(h)))
        return h.value

    def verify(self, h) -> bool:
        """The call's verdict; True when a failed speculation re-ran its pieces."""
        r = C.c_int32()
        check(_lib.load().dml_prereduce_verify(C.c_void_p(h), C.byref(r)))
        return bool(r.value)

    def moments_piece(self, h, block: int, stride: int, off: int, ntask_rows: int, out_ptr: int, stream: int) -> None:
        check(_lib.load().dml_prereduce_moments_piece(C.c_void_p(h), block, stride, off, ntask_rows,
                                                      C.c_void_p(out_ptr), C.c_void_p(stream)))

    def apply_moments(self, store: DataStore, src_ptr: int, rows: int) -> None:
        check(_lib.load().dml_store_apply_adagrad_moments_device(store._h, C.c_void_p(src_ptr), rows), store)

    def stream_wait(self, h, stream: int) -> None:
        check(_lib.load().dml_prereduce_stream_wait(C.c_void_p(h), C.c_void_p(stream)))

    def split(self, fmt: DataDesc, cols: int, total_rows: int, world: int, dev_ptrs: Sequence[int],
              lens: Sequence[int], out_ptr: int, out_cap: int, stream: int) -> List[List[int]]:
        """dml_shard_split: counts[b][d] records of push b for shard d, written dest-major to out."""
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        cnt = (C.c_int64 * max(n * world, 1))()
        check(_lib.load().dml_shard_split(C.byref(fmt.to_c()), cols, total_rows, world, ptrs, ls, n,
                                          C.c_void_p(out_ptr), out_cap, cnt, C.c_void_p(stream)))
        return [[cnt[b * world + d] for d in range(world)] for b in range(n)]


class ShardGroup:
    def __init__(self, fmt: DataDesc, total_rows: int, cols: int, rank: int, world: int,
                 device: Optional[int] = None, ops=None, store_factory=None, pieces: int = 1,
                 reduce_scatter=None, exchange_only: bool = False, emulate_world: int = 0,
                 emulate_channels: int = 32):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.fmt, self.cols, self.rank, self.world = fmt, cols, rank, world
        self.parts: List[KeyRange] = KeyRange(0, total_rows - 1).linearSplit(world)
        self.shard = self.parts[rank]
        self.step_rows = self.parts[0].size()  # linearSplit step: equal padded chunk per rank
        self.total_rows = total_rows
        self.device = device
        self.ops = ops or HipOps()
        # reduce_scatter(out, inp): out = this rank's chunk of sum-over-ranks(inp); runs on the
        # current stream context. Default: RCCL ncclReduceScatter (backend "nccl"), or a
        # host all_reduce + slice under gloo (no reduce_scatter there).
        self._rs = reduce_scatter or self._default_reduce_scatter
        self.store = (store_factory or (lambda: DataStore(fmt, self.shard, cols, device=device)))()
        self.dtype = {0: torch.int32, 1: torch.float32, 3: torch.float64}[fmt.valueType]
        dev = torch.device("cuda", device) if device is not None else torch.device("cpu")
        # exchange_only: a group that only runs push_exchange / push_local (AdaGrad,
        # int32 with intermediate checks) holds no full-model partial buffers
        self.exchange_only = exchange_only
        self.partial = torch.empty(0 if exchange_only else world * self.step_rows * cols, dtype=self.dtype, device=dev)
        self.recv = torch.empty(0 if exchange_only else self.step_rows * cols, dtype=self.dtype, device=dev)
        # pipelining of the full-range path: P row slices, reduce-scattered on a comm stream;
        # calls alternate between two partial/recv buffer sets so call k+1's key index
        # (side stream) and pre-reduce overlap call k's reduce-scatter and apply. P = 1 by
        # default: across calls the reduce-scatter already runs under the next call's
        # pre-reduce, and one launch per call has no per-piece tails (world 1, config 2:
        # 0.441 ms/step against 0.460 for P = 4 and 0.461 for P = 2)
        self.pieces = pieces
        # diagnostic (bench.py --emulate-rs, world 1 only): replace the local shortcut by
        # the HBM footprint an N-rank call has at its owner — a RING reduce-scatter of
        # every piece on the comm stream (N - 1 steps, each reading one 1/N chunk of the
        # partial and the chunk that arrived and writing their sum where the next rank's
        # write would land; dml_diag_ring_rs, on `emulate_channels` blocks as RCCL runs one
        # block per channel), then the apply of 1/N of the shard. The shard's values are
        # then NOT the reduce's result. emulate_world -1: neither (the pieces alone)
        if emulate_world and (world != 1 or (emulate_world > 1 and (self.shard.size() // pieces) % emulate_world)):
            raise ValueError("emulate_world needs world 1 and piece rows divisible by it")
        self.emulate_world = emulate_world
        self.emulate_channels = emulate_channels
        self._landing = None
        self._pending: list = []  # (pre-reduce handle, buffer set) not yet reduce-scattered / checked
        self._pctx = None         # speculative pre-reduce context (dml_prectx), created on first use
        self._xbufs: list = []    # exchange buffers the store may still read: (event, recv, send, push seq)
        self._xpool: list = []    # exchange buffers the store has passed: reused by the next calls
        self._held = None         # the last exchange call's slices, handed to the store next call / flush
        self._k = 0
        if self.partial.is_cuda:
            self.comm = torch.cuda.Stream(device=dev)
            self.cstream = torch.cuda.Stream(device=dev)  # pre-reduce pieces
            self._ready = torch.cuda.Event()
            # high priority: a HIP stream of another priority class gets its own hardware
            # queue, so the next call's index never queues behind this call's pieces
            self.istream = torch.cuda.Stream(device=dev, priority=-1)
            self._partials = [self.partial, torch.empty_like(self.partial)]
            self._recvs = [self.recv, torch.empty_like(self.recv)]
            self._rs_done = [torch.cuda.Event(), torch.cuda.Event()]
            self._applied = [torch.cuda.Event(), torch.cuda.Event()]
            self._store_stream = (torch.cuda.ExternalStream(self.store.stream(), device=dev)
                                  if hasattr(self.store, "stream") else None)

    def _local_rs(self) -> bool:
        """World 1 with the default reduce-scatter: a copy of the partial, skipped."""
        return self.world == 1 and self._rs == self._default_reduce_scatter

    def _default_reduce_scatter(self, out, inp) -> None:
        dist = self.dist
        if self.world == 1:
            out.copy_(inp)
        elif dist.get_backend() == "gloo":
            host = inp.cpu() if inp.is_cuda else inp.clone()
            dist.all_reduce(host)
            n = out.numel()
            out.copy_(host[self.rank * n:(self.rank + 1) * n])
        else:
            dist.reduce_scatter_tensor(out, inp)

    def push_full_range(self, dev_ptrs: Sequence[int], lens: Sequence[int], stream: int = 0) -> None:
        """Ordered local pre-reduce -> reduce-scatter -> owner apply (see module doc)."""
        torch = self.torch
        if self.exchange_only:
            raise RuntimeError("push_full_range on an exchange_only ShardGroup (no partial buffers)")
        if getattr(self, "_held", None) is not None:  # an exchange call's slices come first (call order)
            if self.partial.is_cuda:
                torch.cuda.current_stream(self.partial.device).synchronize()
            self._hand_over()
        if (self.partial.is_cuda and hasattr(self.ops, "begin_ctx") and len(dev_ptrs) <= 64
                and self.step_rows % self.pieces == 0):
            return self._push_pipelined(dev_ptrs, lens)
        if self.partial.is_cuda:
            # the one-shot path reuses buffer set 0: drain the pipelined calls that may still use it,
            # and let the store's stream finish the owner applies that read partial / recv
            # (a previous call's, pipelined or one-shot) before they are rewritten
            self._drain()
            if self._store_stream is not None:
                self._store_stream.synchronize()
        # rows past the matrix end (linearSplit's last shard may be short) stay zero
        self.ops.prereduce(self.fmt, 0, self.total_rows, self.cols, dev_ptrs, lens,
                           self.partial.data_ptr(), stream)
        recv = self.partial if self._local_rs() else self.recv
        if recv is not self.partial:
            self._rs(recv, self.partial)
        if recv.is_cuda:
            torch.cuda.current_stream().synchronize()
        n = self.shard.size() * self.cols
        self.ops.apply(self.store, recv.data_ptr(), n)

    def _push_pipelined(self, dev_ptrs, lens) -> None:
        """Pre-reduce in `pieces` row slices; slice j holds rows [q*S + j*S/P, q*S + (j+1)*S/P)
        of every rank q, laid out [rank][row].

        Speculative and asynchronous across calls (dml_prectx):
        full-range pushes whose records are rows in order, or the permutations a
        call three before listed, skip the key index (side stream) and the pieces
        verify every record. The NEXT call (or flush()) reads this call's verdict —
        a failure re-runs its pieces exactly — and only then reduce-scatters its
        partial on the communication stream, under that next call's pieces; the
        owner apply is queued on the store's stream behind it. Key / repeated-row
        errors are raised by the next call or flush() (like DML_FLAG_ASYNC)."""
        torch = self.torch
        S, P, cols, world = self.step_rows, self.pieces, self.cols, self.world
        blk = S // P
        k = self._k
        self._k ^= 1
        # the key index (side stream) orders after whatever the caller's current stream
        # has enqueued (the producers of the pushes); the pieces run on the group's own
        # stream once the host has seen that index finish (dml_prereduce_piece waits for
        # it), so they follow the producers too — without a cross-stream barrier packet
        # ahead of them on the piece stream (~5 µs between two calls' pieces, measured)
        self._ready.record(torch.cuda.current_stream())
        self.istream.wait_event(self._ready)
        st = self.cstream.cuda_stream
        partial = self._partials[k]
        if self._pctx is None:
            self._pctx = self.ops.ctx_create(self.fmt, 0, self.total_rows, cols, self.device)
        h, local = None, None
        try:
            h = self.ops.begin_ctx(self._pctx, dev_ptrs, lens, self.istream.cuda_stream)
            # buffer set k was last used two calls ago: its apply (queued behind its
            # reduce-scatter) has finished with recv[k], and so has the scatter with partial[k]
            self._applied[k].synchronize()
            for j in range(P):
                piece = partial[j * world * blk * cols:(j + 1) * world * blk * cols]
                self.ops.piece(h, blk, S, j * blk, world * blk, piece.data_ptr(), st)
        except Exception as e:
            # a call that fails here (begin: not whole records, a fourth outstanding call;
            # a piece) still takes its place in the collective sequence: _finish
            # contributes zeros for it and raises e (as dml_group_push_full_range)
            if h is not None:
                self.ops.end(h)
                h = None
            local = e
        self._pending.append((h, k, local))
        err = None
        try:
            self._end_pending(keep=1)  # the previous call: verdict, reduce-scatter, apply, errors
        except Exception as e:
            err = e
        if local is not None:
            try:
                self._end_pending(keep=0)  # this call's zeros, its failure raised now
            except Exception as e:
                err = err or e
        if err is not None:
            raise err

    def _finish(self, h, k, local=None) -> None:
        """A pending call: verdict (exact re-run if the speculation failed), its slices'
        reduce-scatter on the communication stream, the owner apply, its errors.
        `local`: the call already failed before its pieces were recorded (h is None)."""
        torch = self.torch
        S, P, cols, world = self.step_rows, self.pieces, self.cols, self.world
        blk = S // P
        try:
            partial, recv = self._partials[k], self._recvs[k]
            if self._local_rs():
                # one rank: the [rank][row] slices are the shard's rows in order, so
                # the reduce-scatter is the identity and the apply reads the partial
                recv = partial
            failed = local
            if failed is None:
                try:
                    self.ops.verify(h)
                    self.ops.stream_wait(h, self.comm.cuda_stream)  # the pieces (or their re-run)
                except Exception as e:
                    failed = e
            if failed is not None:
                # every rank runs the same collectives whatever fails locally:
                # this rank contributes zeros, skips its apply and raises afterwards. The
                # zeros go in after the pieces and any re-run of them and after
                # the apply of the call two back, which may still read recv[k]
                if h is not None:
                    try:
                        self.ops.stream_wait(h, self.comm.cuda_stream)
                    except Exception:
                        pass
                self.cstream.synchronize()
                self.comm.wait_event(self._applied[k])
                with torch.cuda.stream(self.comm):
                    partial.zero_()
            with torch.cuda.stream(self.comm):
                for j in range(P if recv is not partial else 0):
                    self._rs(recv[j * blk * cols:(j + 1) * blk * cols],
                             partial[j * world * blk * cols:(j + 1) * world * blk * cols])
            if failed is not None:
                # no apply: the set's next use (two calls on) waits for the scatter instead
                self._rs_done[k].record(self.comm)
                self._applied[k].record(self.comm)
                raise failed
            if self.emulate_world < 0:
                self._rs_done[k].record(self.comm)
                return
            if self.emulate_world > 1:
                E = self.emulate_world
                nper = blk * cols // E  # one emulated rank's chunk of a piece
                n = P * nper            # its rows of the whole call
                recv = self._recvs[k]
                if self._landing is None:
                    self._landing = torch.empty(2 * nper, dtype=partial.dtype, device=partial.device)
                esz = partial.element_size()
                for j in range(P):
                    check(_lib.load().dml_diag_ring_rs(
                        self.fmt.valueType, C.c_void_p(partial.data_ptr() + j * blk * cols * esz),
                        C.c_void_p(recv.data_ptr() + j * nper * esz), C.c_void_p(self._landing.data_ptr()),
                        nper * esz, E, 0, self.emulate_channels, C.c_void_p(self.comm.cuda_stream)))
                self._rs_done[k].record(self.comm)
                if not hasattr(self, "_emu_rows"):
                    self._emu_rows = torch.zeros(n, dtype=partial.dtype, device=partial.device)
                with torch.cuda.stream(self._store_stream):  # the 1/N owner apply's bytes
                    self._store_stream.wait_event(self._rs_done[k])
                    self._emu_rows.add_(recv[:n])
                self._applied[k].record(self._store_stream)
                return
            self._rs_done[k].record(self.comm)
            if self._store_stream is not None:
                self._store_stream.wait_event(self._rs_done[k])
            else:
                self.comm.synchronize()
            self.ops.apply(self.store, recv.data_ptr(), self.shard.size() * cols)
            if self._store_stream is not None:
                self._applied[k].record(self._store_stream)
        finally:
            if h is not None:
                self.ops.end(h)

    def _end_pending(self, keep: int = 0) -> None:
        """Finish the oldest calls until `keep` remain, every one of them even when one
        raises (each still issues its collectives, as dml_group's end_pending); the
        first error is raised after them."""
        err = None
        while len(self._pending) > keep:
            try:
                self._finish(*self._pending.pop(0))
            except Exception as e:
                err = err or e
        if err is not None:
            raise err

    def prereduce_stats(self, reset: bool = False) -> dict:
        """dml_prectx_stats of the speculative pre-reduce (identity / reused / indexed pushes)."""
        return self.ops.ctx_stats(self._pctx, reset) if self._pctx is not None else {}

    def record_stride(self) -> int:
        f = self.fmt
        return f.keySize + (f.valueSize * self.cols if f.dataType == DataDesc.DATA_TYPE_MATRIX else f.valueSize)

    def push_exchange(self, dev_ptrs: Sequence[int], lens: Sequence[int]) -> None:
        """Bit-exact path for pushes whose sum does not commute with the store's
        update (AdaGrad, int32 negativity checks) or that hold key subsets: the
        reference's own data flow. Each local push is split by owner shard
        (SparseMatrix.push's per-partition split, SparseMatrix.java:46-60;
        dml_shard_split), the slices go to their owners in one all-to-all (RCCL
        send/recv over xGMI), and every owner applies its W slices in global push
        order — rank-major: rank 0's pushes, then rank 1's — through the store's
        ordered reduce (exact, errors included). Every rank passes the same number
        of pushes per call; keys outside the matrix are dropped like the client does.

        Pipelined over calls: a call's received slices reach the store at the next
        exchange call (once its count exchange, queued behind the previous data
        exchange, has completed) or at flush(), so this call's split overlaps the
        previous all-to-all and the store's apply overlaps this call's all-to-all.
        The push buffers follow the module's contract (allocated and unmodified until
        flush()): at world 1 with every key inside the matrix they go to the store as they
        are, since the split would copy each push whole and nothing crosses a link."""
        torch, dist = self.torch, self.dist
        n, world = len(dev_ptrs), self.world
        stride = self.record_stride()
        self._end_pending(0)  # full-range calls still waiting for their reduce-scatter come first
        dev = self.partial.device
        if world == 1 and n and self.partial.is_cuda and self._whole_shard(dev_ptrs, lens, stride):
            # one owner and every key inside the matrix: the split would copy each push
            # whole and nothing crosses a link, so the store takes the pushes themselves
            # (they stay allocated and unmodified until flush(), the module's contract)
            self._hand_over()
            self.store.pushDevice(list(dev_ptrs), list(lens))
            return
        cap = int(sum(lens))
        send = self._xalloc(max(cap, 1), dev)
        st = torch.cuda.current_stream(dev).cuda_stream if send.is_cuda else 0
        counts = self.ops.split(self.fmt, self.cols, self.total_rows, world, list(dev_ptrs), list(lens),
                                send.data_ptr(), cap, st) if n else []
        mine = torch.tensor([[counts[b][d] for b in range(n)] for d in range(world)], dtype=torch.int64)
        theirs = torch.empty_like(mine)  # [source rank][its push b]
        # gloo has no device all-to-all: host copies (CPU tests, ranks sharing one GPU)
        host_a2a = world > 1 and (not send.is_cuda or dist.get_backend() == "gloo")
        if world == 1:
            theirs.copy_(mine)
        elif host_a2a:
            dist.all_to_all_single(theirs.view(-1), mine.view(-1))
        else:
            t = theirs.to(dev)
            dist.all_to_all_single(t.view(-1), mine.to(dev).view(-1))
            theirs = t.cpu()  # waits for the previous call's data exchange too (same stream)
        if send.is_cuda:
            torch.cuda.current_stream(dev).synchronize()
        self._hand_over()  # the previous call's slices have arrived
        send_sizes = [int(mine[d].sum()) * stride for d in range(world)]
        recv_sizes = [int(theirs[q].sum()) * stride for q in range(world)]
        nsend, nrecv = sum(send_sizes), sum(recv_sizes)
        if world == 1:
            recv = send  # the one owner: the split's owner-major layout is the receive layout
        elif host_a2a and send.is_cuda:
            recv = self._xalloc(max(nrecv, 1), dev)
            hr = torch.empty(nrecv, dtype=torch.uint8)
            dist.all_to_all_single(hr, send[:nsend].cpu(), recv_sizes, send_sizes)
            recv[:nrecv].copy_(hr)
        else:
            recv = self._xalloc(max(nrecv, 1), dev)
            dist.all_to_all_single(recv[:nrecv], send[:nsend], recv_sizes, send_sizes)
        ptrs, ls, off = [], [], 0
        for q in range(world):
            for b in range(n):
                ln = int(theirs[q][b]) * stride
                if ln:
                    ptrs.append(recv.data_ptr() + off)
                    ls.append(ln)
                off += ln
        # held until the next call / flush; `send` stays alive until the exchange ran
        self._held = (ptrs, ls, recv, send)

    def push_moments(self, dev_ptrs: Sequence[int], lens: Sequence[int], stream: int = 0) -> None:
        """AdaGrad's sharded path for many pushes per rank:
        the rank's full-range pushes pre-reduced into Σu and Σu² per element (one
        [row][Σu | Σu²] partial), one reduce-scatter of both, and the owner's
        row += Σu, delta += Σu², alpha = f(final delta)
        (dml_store_apply_adagrad_moments_device). xGMI bytes per rank stay
        (world-1)/world x 2 x the model whatever the pushes per rank; results are
        within 1e-6 of the sequential reference, not bit-exact (push_exchange is).
        Index errors surface at the next call or flush()."""
        torch = self.torch
        if not self.fmt.adaGrad:
            raise ValueError("push_moments is the AdaGrad path (push_full_range sums plain matrices)")
        self._hand_over()
        self._end_pending(0)
        S, world, cols = self.step_rows, self.world, self.cols
        dev = torch.device("cuda", self.device) if self.device is not None else torch.device("cpu")
        if not hasattr(self, "_mparts"):
            self._mparts = [torch.empty(world * S * 2 * cols, dtype=torch.float32, device=dev) for _ in range(2)]
            self._mrecvs = [torch.empty(S * 2 * cols, dtype=torch.float32, device=dev) for _ in range(2)]
            self._m_applied = [torch.cuda.Event(), torch.cuda.Event()]
            self._mpending = []
            self._mk = 0
        k = self._mk
        self._mk ^= 1
        self._ready.record(torch.cuda.current_stream())
        self.cstream.wait_event(self._ready)
        self.istream.wait_event(self._ready)
        h = self.ops.begin(self.fmt, 0, self.total_rows, cols, list(dev_ptrs), list(lens), self.istream.cuda_stream)
        self._m_applied[k].synchronize()  # set k's last apply (two calls ago) is done
        part, recv = self._mparts[k], self._mrecvs[k]
        try:
            self.ops.moments_piece(h, S, S, 0, world * S, part.data_ptr(), self.cstream.cuda_stream)
            self.ops.stream_wait(h, self.comm.cuda_stream)
            with torch.cuda.stream(self.comm):
                self._rs(recv, part)
            done = torch.cuda.Event()
            done.record(self.comm)
            if self._store_stream is not None:
                self._store_stream.wait_event(done)
            else:
                self.comm.synchronize()
            self.ops.apply_moments(self.store, recv.data_ptr(), self.shard.size())
            if self._store_stream is not None:
                self._m_applied[k].record(self._store_stream)
        except BaseException:
            self.ops.end(h)
            raise
        self._mpending.append(h)
        while len(self._mpending) > 1:  # the previous call's index errors
            self.ops.end(self._mpending.pop(0))

    def _whole_shard(self, dev_ptrs, lens, stride) -> bool:
        """World 1: every record's key lies in [0, total_rows) (dml_shard_split, counts only)."""
        st = self.torch.cuda.current_stream(self.partial.device).cuda_stream
        counts = self.ops.split(self.fmt, self.cols, self.total_rows, 1, list(dev_ptrs), list(lens), 0, 0, st)
        return all(counts[b][0] * stride == int(lens[b]) for b in range(len(lens)))

    def _hand_over(self) -> None:
        """Push the last exchange call's received slices into the store (asynchronous
        apply); their buffers stay alive until the store has read them."""
        held, self._held = getattr(self, "_held", None), None
        if held is None:
            return
        ptrs, ls, recv, send = held
        if ptrs:
            self.store.pushDevice(ptrs, ls)
        if not recv.is_cuda:
            return  # host stand-in stores apply synchronously
        if getattr(self, "_store_stream", None) is None:
            self.torch.cuda.synchronize(recv.device)
            return
        ev = self.torch.cuda.Event()
        ev.record(self._store_stream)
        seq = self.store.push_seq()
        # keep the buffers until the store has passed them: its stream's reads (the
        # event) and its host-side retire of those chunks, which may read the pushes
        # again (exact replay, int32 rollback, re-run of a failed speculation);
        # passed ones go back to the pool the next calls allocate from (no allocator
        # churn on GB buffers)
        keep = []
        for x in self._xbufs:
            if x[0].query():
                self._xpass(x)
            else:
                keep.append(x)
        keep.append((ev, recv, send, seq))
        while len(keep) > 3:  # bound the memory held for the asynchronous store
            x = keep.pop(0)
            x[0].synchronize()
            self._xpass(x)
        self._xbufs = keep

    def _xpass(self, x) -> None:
        """Release an exchange buffer set once the store has retired the call that read it."""
        self.store.retire(x[3])
        self._xrelease(x[1], x[2])

    def _xalloc(self, n: int, dev):
        """An exchange buffer of at least n bytes: the smallest free pooled one, or new."""
        keep = []
        for x in self._xbufs:  # buffers the store has passed since the last hand-over
            if x[0].query():
                self._xpass(x)
            else:
                keep.append(x)
        self._xbufs = keep
        fit = [t for t in self._xpool if t.numel() >= n]
        if fit:
            t = min(fit, key=lambda x: x.numel())
            self._xpool = [x for x in self._xpool if x is not t]  # by identity (tensor == is elementwise)
            return t
        return self.torch.empty(n, dtype=self.torch.uint8, device=dev)

    def _xrelease(self, *bufs) -> None:
        for t in bufs:
            if all(t is not u for u in self._xpool):
                self._xpool.append(t)
        while len(self._xpool) > 2:  # keep the largest two (a send and a receive buffer)
            small = min(self._xpool, key=lambda x: x.numel())
            self._xpool = [x for x in self._xpool if x is not small]

    def push_local(self, dev_ptrs: Sequence[int], lens: Sequence[int]) -> None:
        """Pushes already split to this shard: exact ordered apply, no exchange — after
        every earlier group call's apply (the store applies calls in call order).
        Reads of `self.store` between calls see only what was applied: flush() first."""
        if getattr(self, "_held", None) is not None:
            if self.partial.is_cuda:
                self.torch.cuda.current_stream(self.partial.device).synchronize()
            self._hand_over()
        self._end_pending(0)
        self.store.pushDevice(dev_ptrs, lens)

    def _drain(self) -> None:
        """Every pipelined call's pieces, reduce-scatters and applies have finished."""
        try:
            if getattr(self, "_held", None) is not None:
                if self.partial.is_cuda:
                    self.torch.cuda.current_stream(self.partial.device).synchronize()
                self._hand_over()
            self._end_pending(0)
            while getattr(self, "_mpending", None):
                self.ops.end(self._mpending.pop(0))
        finally:
            if self.partial.is_cuda:
                self.istream.synchronize()
                self.cstream.synchronize()
                self.comm.synchronize()
                for ev in self._applied:
                    ev.synchronize()

    def flush(self):
        """Every pushed call applied; raises the first deferred pre-reduce error."""
        try:
            self._drain()
        finally:
            self.store.flush()
            self._xbufs.clear()
            self._xpool.clear()

    def close(self) -> None:
        """Flush, then release the shard store and the partial / receive buffers."""
        try:
            self.flush()
        finally:
            if self._pctx is not None:
                self.ops.ctx_destroy(self._pctx)
                self._pctx = None
            self.store.close()
            self._partials = self._recvs = []
            self.partial = self.recv = None
            self._xbufs.clear()


class NativeShardGroup:
    """The same sharded path through the C-ABI's own RCCL communicator
    (dml_group_*, distml_amd/csrc/dml_group.hip): what a host without
    torch.distributed (the JNI deployment) binds. `unique_id` is the 128 bytes
    NativeShardGroup.unique_id() returns on rank 0, distributed by the caller."""

    def __init__(self, fmt: DataDesc, total_rows: int, cols: int, rank: int, world: int, unique_id: bytes,
                 device: int = 0, pieces: int = 1):
        L = _lib.load()
        self._L = L
        if len(unique_id) != 128:
            raise ValueError("unique_id must be the 128 bytes of NativeShardGroup.unique_id()")
        h = C.c_void_p()
        idb = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        check(L.dml_group_create(idb, world, rank, device, C.byref(fmt.to_c()), total_rows, cols, pieces,
                                 C.byref(h)))
        self._h = h.value
        self.fmt, self.cols, self.rank, self.world = fmt, cols, rank, world
        self.shard = KeyRange(0, total_rows - 1).linearSplit(world)[rank]
        sp = C.c_void_p()
        check(L.dml_group_store(C.c_void_p(self._h), C.byref(sp)))
        self.store = DataStore._wrap(fmt, self.shard, cols, device, sp.value)

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        check(_lib.load().dml_group_unique_id(buf, 128))
        return bytes(buf)

    def push_full_range(self, dev_ptrs: Sequence[int], lens: Sequence[int]) -> None:
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        check(self._L.dml_group_push_full_range(C.c_void_p(self._h), ptrs, ls, n))

    def push_moments(self, dev_ptrs: Sequence[int], lens: Sequence[int]) -> None:
        """The two-moment AdaGrad path (dml_group_push_moments), within 1e-6."""
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        check(self._L.dml_group_push_moments(C.c_void_p(self._h), ptrs, ls, n), self.store)

    def push_local(self, dev_ptrs: Sequence[int], lens: Sequence[int]) -> None:
        """Pushes already split to this shard (dml_group_push_local): the exact ordered
        apply, after every earlier group call's."""
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        check(self._L.dml_group_push_local(C.c_void_p(self._h), ptrs, ls, n), self.store)

    def debug_fail_verify(self, nth: int) -> None:
        """Fault injection (tests): the nth full-range call finished from now fails its verdict."""
        check(self._L.dml_group_debug_fail_verify(C.c_void_p(self._h), nth))

    def push_exchange(self, dev_ptrs: Sequence[int], lens: Sequence[int]) -> None:
        """The exact split / all-to-all / ordered-owner-apply path (dml_group_push_exchange)."""
        n = len(dev_ptrs)
        ptrs = (C.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (C.c_int64 * max(n, 1))(*lens)
        check(self._L.dml_group_push_exchange(C.c_void_p(self._h), ptrs, ls, n), self.store)

    def flush(self) -> None:
        check(self._L.dml_group_flush(C.c_void_p(self._h)), self.store)

    def prereduce_stats(self, reset: bool = False) -> dict:
        c = _lib.dml_store_counters()
        check(self._L.dml_group_prereduce_stats(C.c_void_p(self._h), C.byref(c), int(reset)))
        return {f: getattr(c, f) for f, _ in c._fields_}

    def close(self) -> None:
        if self._h:
            self.store._h = None  # owned by the group
            self._L.dml_group_destroy(C.c_void_p(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
