"""Query Sample Library and Offline SUT over the HIP engine.

Mirrors the reference's LoadGen-facing surface (the real MLPerf LoadGen is not installable
offline, so the query / response types are plain Python):
  * QSLs (csrc/rnnt_qsl.{hpp,cpp} / models/rnnt_qsl.py): per-sample features and lengths;
    ``sort`` is the length-descending bucket sort (rnnt_qsl.cpp:104-133); ``batch_inputs`` is
    AssembleSamples (rnnt_qsl.cpp:150-188) -- for the HBM-resident ``GpuQSL`` it hands the engine
    the ragged store and the batch's row offsets, which the engine gathers inside its quantize pass.
  * ``OfflineSUT`` (csrc/torch_sut.cpp:88-236 / models/pytorch_sut.py:58-118): issue_queries sorts
    the query, splits it into batches and runs them through its engines -- one host thread per
    engine pulling batches from one shared work list (the reference's INTER worker threads pulling
    from one queue, torch_sut.cpp:143-182) -- and completes every sample with its int32 token row
    (QuerySamplesComplete, torch_sut.cpp:221-236) through one completion point.  Engines may sit on
    several GPUs of the process (one stream per engine on its own device; encoders on one device
    take turns, so each batch's latency-bound greedy decode overlaps the next batch's encoder).
Multi-process (one process per GPU, bench.py / rnnt_amd.dist): every rank sorts the same query
into the same batches and claims them from one shared counter (``dist.BatchClaim``, passed to
``OfflineSUT.issue_batches``) whenever its encoder is free, and the responses are streamed to rank
0's host (``dist.ResponseStream``).
"""
import collections
import threading
from dataclasses import dataclass

import numpy as np

from .config import RNNTParam as R
from .engine import pad_batch


@dataclass
class QuerySample:
    id: int
    index: int


class _SortedQSL:
    def __len__(self):
        return self.count

    def sort_indices(self, indices):
        """Positions of `indices` in longest-first order, stable (the bucket sort's order).  The key
        is the length's distance from the longest as uint16, which numpy's stable sort orders by
        radix sort (O(n): 196k query samples at 8 GPUs in ~5 ms instead of ~20)."""
        lens = self.lengths[np.asarray(indices, np.int64)]
        if len(lens) and int(self.lengths.max()) - int(self.lengths.min()) < 65536:
            return np.argsort((np.int64(self.lengths.max()) - lens).astype(np.uint16), kind="stable")
        return np.argsort(-lens, kind="stable")

    def sort(self, samples, reverse=True):
        """Bucket sort by feature length, longest first (rnnt_qsl.cpp:104-133)."""
        lmin, lmax = int(self.lengths.min()), int(self.lengths.max())
        buckets = [[] for _ in range(lmax - lmin + 1)]
        for s in samples:
            L = int(self.lengths[s.index])
            buckets[(lmax - L) if reverse else (L - lmin)].append(s)
        return [s for b in buckets for s in b]


class RNNTQSL(_SortedQSL):
    def __init__(self, features, lengths):
        """features: list of [T_i, 240] float32 arrays (or None for synthetic on-demand);
        lengths: int array [count]."""
        self.lengths = np.asarray(lengths, np.int32)
        self.features = features
        self.count = len(self.lengths)

    @classmethod
    def synthetic(cls, lengths, seed):
        rng = np.random.default_rng(seed)
        feats = [rng.standard_normal((int(l), R.trans_input_size), dtype=np.float32) for l in lengths]
        return cls(feats, lengths)

    def assemble(self, indices, n_pad=None):
        """-> (x [T_max, n_pad, 256] f32, lens [n_pad] int32), zero padded (rnnt_qsl.cpp:150-188)."""
        n = len(indices)
        n_pad = n_pad or pad_batch(n)
        lens = np.zeros(n_pad, np.int32)
        lens[:n] = self.lengths[list(indices)]
        T = int(lens.max())
        x = np.zeros((T, n_pad, R.PADDED_INPUT_SIZE), np.float32)
        for i, idx in enumerate(indices):
            f = self.features[idx]
            x[: f.shape[0], i, : R.trans_input_size] = f
        return x, lens

    def batch_inputs(self, indices, n_pad, device):
        import torch
        x, lens = self.assemble(indices, n_pad)
        return dict(x=torch.from_numpy(x).to(device), lens=torch.from_numpy(lens).to(device),
                    lens_host=lens[: len(indices)], T=x.shape[0])


def batch_bounds(n, batch, sizes=None):
    """Start/end of each batch over a sorted query: ``sizes`` (the last entry repeats) or uniform
    ``batch``."""
    out, i, k = [], 0, 0
    while i < n:
        b = sizes[min(k, len(sizes) - 1)] if sizes else batch
        out.append((i, min(n, i + b)))
        i += b
        k += 1
    return out


def make_batches(qsl, ids, idx, batch_size, sizes=None):
    """An Offline query (sample ids, QSL indices) sorted longest first (rnnt_qsl.cpp:104-133) and
    split into batches: a list of (ids, idx) array pairs."""
    order = qsl.sort_indices(idx)
    ids, idx = np.asarray(ids, np.int64)[order], np.asarray(idx, np.int64)[order]
    return [(ids[i:e], idx[i:e]) for i, e in batch_bounds(len(ids), batch_size, sizes)]


class OfflineSUT:
    def __init__(self, engines, qsl, batch_size=1024, batch_sizes=None, on_complete=None, early_decodes=None):
        """engines: one Engine or a list (several per GPU keep batches in flight; engines on
        different devices serve one query together).  qsl: one QSL, or {device: QSL} when each
        GPU holds its own copy of the samples (GpuQSL replicas).  early_decodes: None = every
        batch decodes right after its encode (beside the next batch's encoder); k = when the query
        has no more batches than engines, only the first k batches do, the others' decodes wait
        until every encode is done (they then run beside each other, not beside an encoder)."""
        self.early_decodes = early_decodes
        self.engines = list(engines) if isinstance(engines, (list, tuple)) else [engines]
        self.engine = self.engines[0]
        self.qsl, self.batch_size, self.batch_sizes = qsl, batch_size, batch_sizes
        self.on_complete = on_complete
        self.on_batch = None  # called with (ids, lens, tokens) of every completed batch
        self._done_lock = threading.Lock()
        self.completed = []  # per batch: (sample ids int64 [n], lengths int32 [n], tokens int32 [sum])
        self._streams = {}
        self._enc_turns = {}  # device -> (Condition, deque of batch indices in encode order)
        self._gates = {}  # device -> Lock held from a shared-list claim to the end of that batch's encode
        self.encode_order = []  # batch indices in the order their encodes ran (all devices)
        self._hold = None

    def qsl_for(self, device):
        return self.qsl[device] if isinstance(self.qsl, dict) else self.qsl

    def issue_queries(self, samples):
        """LoadGen's IssueQuery: sort the query longest first, batch it, run it."""
        ids = np.fromiter((s.id for s in samples), np.int64, len(samples))
        idx = np.fromiter((s.index for s in samples), np.int64, len(samples))
        self.issue_batches(make_batches(self.qsl_for(self.engine.device), ids, idx, self.batch_size, self.batch_sizes))

    def issue_batches(self, batches, claim=None):
        """Run pre-formed batches -- (sample ids, QSL indices) int64 array pairs, each
        length-sorted (make_batches) -- on the engines: one host thread per engine pulls the next
        batch from the shared list.  self.batch_engine[i] records which engine ran batch i (None:
        another process ran it).

        claim: None = this process runs every batch; or a callable returning the next batch index
        of a list shared with other processes (dist.BatchClaim), None once all are taken.  An
        engine thread then claims only when its device's encoder is free (it holds the device's
        encode gate from the claim to the end of that batch's encode), so batches go, longest
        first, to whichever GPU can start them soonest -- the reference's instances pulling from
        one queue (torch_sut.cpp:167-182) across processes."""
        nxt = [0]
        take = threading.Lock()
        errors = []
        self.batch_engine = [None] * len(batches)
        self.encode_order = []
        k = self.early_decodes
        hold = claim is None and k is not None and k < len(batches) <= len(self.engines)
        self._hold = None
        if hold:  # the held batches wait until every batch of the query is encoded (or one encode failed)
            self._hold = dict(k=k, cv=threading.Condition(), done=0, failed=False, nb=len(batches))
        for eng in self.engines:
            self._stream_for(eng)
            self._enc_turns.setdefault(eng.device, (threading.Condition(), collections.deque()))
            self._gates.setdefault(eng.device, threading.Lock())

        def worker(eng):
            try:
                while True:
                    gate = None
                    if claim is None:
                        with take:
                            i = nxt[0]
                            nxt[0] += 1
                            if i < len(batches):  # encoders on one GPU run in batch order (longest first)
                                self._enc_turns[eng.device][1].append(i)
                        if i >= len(batches):
                            return
                    else:
                        gate = self._gates[eng.device]
                        gate.acquire()  # released by _run_batch once this batch is encoded
                        try:
                            i = claim()
                            if i is not None:
                                if not 0 <= i < len(batches):
                                    raise RuntimeError(f"OfflineSUT: claimed batch {i} of {len(batches)}")
                                with take:
                                    self._enc_turns[eng.device][1].append(i)
                        except BaseException:
                            gate.release()
                            raise
                        if i is None:
                            gate.release()
                            return
                    self.batch_engine[i] = self.engines.index(eng)
                    self._run_batch(eng, *batches[i], bi=i, gate=gate)
            except Exception as ex:  # surfaced below: never leave the query half-complete silently
                errors.append(ex)

        if len(self.engines) == 1:
            worker(self.engines[0])
        else:
            ths = [threading.Thread(target=worker, args=(e,)) for e in self.engines]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        if errors:
            raise errors[0]

    def warmup(self, iters=1, batch_size=None, frames=R.MAX_FEA_LEN):
        """OfflineSUT::warmup (torch_sut.cpp:124-138): before the first query, run `iters` batches of
        dummy samples (QSL::GenerateDummySamples, rnnt_qsl.cpp:136-147: N(0,1) features of
        MAX_FEA_LEN frames, every length MAX_FEA_LEN) through every engine -- encode + greedy decode
        on the engine's own stream -- so first-call costs (code-object loads, lazy allocations,
        the engine's workspace first touch) land here, not in the first query.  Nothing is
        completed.  batch_size: rows per dummy batch (default: the SUT's batch size, at most the
        engine's capacity).  -> seconds spent."""
        import time
        t0 = time.perf_counter()
        for eng in self.engines:  # every engine's stream exists before any work is queued (as in issue_batches)
            self._stream_for(eng)
        for eng in self.engines:
            n = max(1, min(int(batch_size or self.batch_size), int(eng.max_batch)))
            n_pad = pad_batch(n)
            dummy = DummyQSL(frames, seed=0)
            st = self._stream_for(eng)
            for _ in range(int(iters)):
                with self._device_scope(eng, st):
                    enc = self._encode(eng, st, None, np.zeros(n, np.int64), n, n_pad, qsl=dummy)
                    self._decode(eng, st, enc)
            del dummy, enc
        _release_cached(self.engines)  # the dummy batches' inputs are transient: give their blocks back
        return time.perf_counter() - t0

    def ran_batches(self, batches):
        """The batches of the last issue_batches call this process ran (all of them without a claim)."""
        return [b for b, e in zip(batches, self.batch_engine) if e is not None]

    # ---- device hooks (a host-only test stands in for these; tests/test_sut_dist.py)
    def _stream_for(self, eng):
        import torch
        if id(eng) not in self._streams:
            self._streams[id(eng)] = torch.cuda.Stream(device=eng.device)
        return self._streams[id(eng)]

    def _device_scope(self, eng, st):
        import contextlib
        import torch
        scope = contextlib.ExitStack()
        scope.enter_context(torch.cuda.device(eng.device))
        scope.enter_context(torch.cuda.stream(st))
        return scope

    def _encode(self, eng, st, ids, idx, n, n_pad, qsl=None):
        """Enqueue and finish one batch's encode; -> the decode's output buffers."""
        import torch
        res = torch.empty((n, eng.max_res), dtype=torch.int32, device=st.device)
        rl = torch.empty(n, dtype=torch.int32, device=st.device)
        inp = (qsl or self.qsl_for(eng.device)).batch_inputs(idx, n_pad, torch.device("cuda", eng.device))
        if "store" in inp:
            eng.encode_gather(inp["store"], inp["offsets"], inp["lens"], inp["lens_host"], inp["T"], n, n_pad, stream=st)
        else:
            eng.encode(inp["x"], inp["lens"], inp["lens_host"], n=n, stream=st)
        st.synchronize()
        return res, rl

    def _decode(self, eng, st, enc):
        """The greedy decode of the encoded batch -> (lengths int32 [n] host, tokens [n, >=max len] host)."""
        res, rl = enc
        eng.decode(res, rl, stream=st)
        rlh = rl.cpu().numpy()
        return rlh, res[:, : max(1, int(rlh.max()))].cpu().numpy()

    def _run_batch(self, eng, ids, idx, bi=0, gate=None):
        """One batch on `eng`: wait for this device's encode turn, encode, hand the turn and the
        encode gate on, decode, complete.  The turn and the gate are handed on exactly once on every
        path -- also when getting the stream, the device scope or the turn wait raises (ADVICE r04:
        a gate held by a failed worker would block the device's other workers forever)."""
        n = len(ids)
        n_pad = pad_batch(n)
        cv, turn = self._enc_turns[eng.device]
        handed = [False]
        encoded = [False]

        def hand_on():
            if handed[0]:
                return
            handed[0] = True
            with cv:
                if turn and turn[0] == bi:
                    turn.popleft()
                else:  # failed before our turn came: drop our place so later batches are not blocked
                    try:
                        turn.remove(bi)
                    except ValueError:
                        pass
                cv.notify_all()
            if gate is not None:  # the device's encoder is free: the next claim may go
                gate.release()
            h = self._hold
            if h is not None:  # counted even when the encode raised, so the held decodes never wait forever
                with h["cv"]:
                    h["done"] += 1
                    h["failed"] = h["failed"] or not encoded[0]
                    h["cv"].notify_all()

        try:
            st = self._stream_for(eng)
            with self._device_scope(eng, st):
                # encoders on one GPU take turns in batch order (longest first): the longest batch's
                # decode overlaps the most encoding, and the last encode is the shortest batch's
                with cv:
                    cv.wait_for(lambda: turn[0] == bi)
                    self.encode_order.append(bi)
                try:
                    enc = self._encode(eng, st, ids, idx, n, n_pad)
                    encoded[0] = True
                finally:
                    hand_on()
                h = self._hold
                if h is not None and bi >= h["k"]:
                    with h["cv"]:
                        h["cv"].wait_for(lambda: h["done"] == h["nb"] or h["failed"])
                        if h["failed"]:
                            raise RuntimeError("OfflineSUT: an encode of this query failed; held decode abandoned")
                rlh, toks = self._decode(eng, st, enc)
        finally:
            hand_on()
        self.query_samples_complete(ids, idx, toks, rlh)

    def query_samples_complete(self, ids, idx, toks, lens):
        """Response = int32 tokens [res_len] per sample (torch_sut.cpp:221-236)."""
        flat = toks[np.arange(toks.shape[1])[None, :] < lens[:, None]]
        if self.on_batch is not None:  # e.g. dist.ResponseStream.push: ship the batch to rank 0 now
            self.on_batch(ids, lens.astype(np.int32), flat.astype(np.int32))
        with self._done_lock:
            self.completed.append((ids, lens.astype(np.int32), flat.astype(np.int32)))
            if self.on_complete:
                off = 0
                for i in range(len(ids)):
                    self.on_complete(QuerySample(id=int(ids[i]), index=int(idx[i])), flat[off: off + lens[i]])
                    off += int(lens[i])

    def take_completed(self):
        """-> (ids int64 [n], lengths int32 [n], tokens int32 [sum]) of every completed sample
        since the last call (the payloads QuerySamplesComplete hands LoadGen)."""
        with self._done_lock:
            done, self.completed = self.completed, []
        if not done:
            return np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32)
        return tuple(np.concatenate([d[k] for d in done]) for k in range(3))

    @property
    def responses(self):
        """{sample id: token row} of the completed samples."""
        out = {}
        with self._done_lock:
            for ids, lens, flat in self.completed:
                off = 0
                for i, L in zip(ids, lens):
                    out[int(i)] = flat[off: off + L].copy()
                    off += int(L)
        return out

    def flush_queries(self):
        pass


def _release_cached(engines):
    """Return the caching allocator's free blocks on the engines' devices (after a warmup's large
    transient dummy inputs) once their streams are idle."""
    import torch
    if not torch.cuda.is_available():  # host-side tests stand in for the devices
        return
    for dev in sorted({e.device for e in engines}):
        with torch.cuda.device(dev):
            torch.cuda.synchronize()
            torch.cuda.empty_cache()


class DummyQSL:
    """QSL::GenerateDummySamples (rnnt_qsl.cpp:136-147) for the SUT warmups: every requested sample
    is the same `frames`-frame N(0,1) feature sample (240 channels, length `frames`), generated on
    the target device and handed over in the gather form of GpuQSL (one sample in a store, every
    row's offset 0) -- the engine's gather-quantize pass assembles the batch, so no dense
    [frames, n_pad, 256] batch is materialised (a dense 4096 x 500-frame dummy
    batch left later queries slower)."""

    def __init__(self, frames=R.MAX_FEA_LEN, seed=0):
        self.frames, self.seed = int(frames), int(seed)

    def batch_inputs(self, indices, n_pad, device=None):
        import torch
        n = len(indices)
        g = torch.Generator(device=device)
        g.manual_seed(self.seed)
        store = torch.randn((self.frames, R.trans_input_size), device=device, generator=g)
        lens = torch.zeros(n_pad, dtype=torch.int32, device=device)
        lens[:n] = self.frames
        return dict(store=store, offsets=torch.zeros(n, dtype=torch.int64, device=device), lens=lens,
                    lens_host=np.full(n, self.frames, np.int32), T=self.frames)


class GpuQSL(_SortedQSL):
    """QSL with every sample's features resident in HBM, ragged ([sum T_i, 240] fp32,
    LoadSamplesToRam); AssembleSamples (rnnt_qsl.cpp:150-188) is the engine's gather-quantize pass
    over this store (rnnt_engine_encode_gather), or ``assemble`` for an explicit padded copy.
    Synthetic N(0,1) features, seeded (the same seed gives the same store on every device)."""

    def __init__(self, lengths, seed, device="cuda", store=None):
        import torch
        self.lengths = np.asarray(lengths, np.int32)
        self.count = len(self.lengths)
        self.offsets = np.concatenate([[0], np.cumsum(self.lengths)[:-1]]).astype(np.int64)
        if store is None:
            g = torch.Generator(device=device)
            g.manual_seed(int(seed))
            store = torch.randn((int(self.lengths.sum()), R.trans_input_size), device=device, generator=g)
        self.feats = store
        self.device = torch.device(device)

    def batch_inputs(self, indices, n_pad, device=None):
        import torch
        idx = np.asarray(indices, np.int64)
        n = len(idx)
        bl = self.lengths[idx].astype(np.int32)
        lp = np.zeros(n_pad, np.int32)
        lp[:n] = bl
        return dict(store=self.feats, offsets=torch.from_numpy(self.offsets[idx]).to(self.device),
                    lens=torch.from_numpy(lp).to(self.device), lens_host=bl, T=max(int(bl.max()), 1))

    def assemble(self, indices, n_pad=None):
        """-> (x cuda [T_max, n_pad, 256] fp32, lens cuda int32 [n_pad], lens_host [n])."""
        import torch
        idx = np.asarray(indices, np.int64)
        n = len(idx)
        n_pad = n_pad or pad_batch(n)
        bl = self.lengths[idx].astype(np.int32)
        lp = np.zeros(n_pad, np.int32)
        lp[:n] = bl
        T = int(bl.max())
        t = torch.arange(T, device=self.device)[:, None]
        ln = torch.from_numpy(bl).to(self.device)[None, :]
        rows = torch.from_numpy(self.offsets[idx]).to(self.device)[None, :] + t
        valid = t < ln
        x = torch.zeros((T, n_pad, R.PADDED_INPUT_SIZE), dtype=torch.float32, device=self.device)
        x[:, :n, : R.trans_input_size] = self.feats[torch.where(valid, rows, 0)] * valid[..., None]
        return x, torch.from_numpy(lp).to(self.device), bl


class GpuWavQSL(_SortedQSL):
    """WAV=true QSL (launch_sut.sh:53-55; AssembleSamples(processor=true) + AudioProcessor,
    rnnt_qsl.cpp:150-188, torch_sut.cpp:192-200): every sample's 16 kHz audio resident in HBM,
    ragged, and ``assemble`` runs the GPU featurizer straight from that storage (per-row
    offsets: no padded [N, max_len] copy) into the engine's [T, n_pad, 256] layout.  One
    featurizer per calling thread (its workspace is per object), on the caller's stream.
    ``lengths`` are the feature lengths (what the SUT sorts by), ``wav_lengths`` the samples."""

    def __init__(self, wavs, device="cuda", featurizer_kwargs=None):
        import torch
        from .featurizer import feature_frames
        self.wav_lengths = np.array([len(w) for w in wavs], np.int32)
        self.lengths = np.array([feature_frames(int(v)) for v in self.wav_lengths], np.int32)
        self.count = len(wavs)
        self.offsets = np.concatenate([[0], np.cumsum(self.wav_lengths.astype(np.int64))[:-1]]).astype(np.int64)
        self.store = torch.cat([torch.as_tensor(w, dtype=torch.float32).to(device) for w in wavs] +
                               [torch.zeros(1, device=device)])
        self.device = device
        self._kw = dict(sample_rate=16000, window="hann", n_fft=512, nfilt=80, frame_splicing=3, pad_out_feat=True)
        self._kw.update(featurizer_kwargs or {})
        self._tls = threading.local()

    def _featurizer(self):
        fz = getattr(self._tls, "fz", None)
        if fz is None:
            import torch
            from .featurizer import FilterbankFeatures
            fz = FilterbankFeatures(device=torch.device(self.device).index or 0, **self._kw)
            self._tls.fz = fz
        return fz

    def assemble(self, indices, n_pad=None):
        """-> (x cuda [T_max, n_pad, 256] fp32, lens cuda int32 [n_pad], lens_host [n])."""
        import torch
        idx = np.asarray(indices, np.int64)
        n = len(idx)
        n_pad = n_pad or pad_batch(n)
        bl = self.lengths[idx].astype(np.int32)
        wl = self.wav_lengths[idx].astype(np.int32)
        off = torch.from_numpy(self.offsets[idx]).to(self.device)
        x, lens = self._featurizer().featurize(self.store, torch.from_numpy(wl).to(self.device), wl, n=n, n_pad=n_pad,
                                               T_out=max(int(bl.max()), 1), offsets=off)
        return x, lens, bl

    def batch_inputs(self, indices, n_pad, device=None):
        x, lens, bl = self.assemble(indices, n_pad)
        return dict(x=x, lens=lens, lens_host=bl, T=x.shape[0])


class FeatureStore:
    """One device's Server feature store: ``slots`` fixed ranges of ``max_frames`` 240-channel fp32
    rows in HBM -- the reference's per-sample processed feature tensors (torch_sut.cpp:454-461, one
    [T][1][C] tensor per sample on mProcessedQueue_) kept resident instead.  A producer featurizes
    an arriving sample into a free slot (rnnt_featurizer_run_rows), the engines of its lane encode
    it from there chunk by chunk (rnnt_engine_encode_stream, offset = slot row + position) and the
    slot is released once the sample's last chunk is encoded.  Fixed slots (O(1) alloc / release,
    no fragmentation): 2048-slot stores of 35 s samples are ~2 GB, small beside 288 GB of HBM.
    The free list is host-side; ``alloc=False`` keeps the bookkeeping alone (CPU tests)."""

    def __init__(self, slots, max_frames, device="cuda", alloc=True):
        if int(slots) <= 0 or int(max_frames) <= 0:
            raise ValueError("a feature store needs slots > 0 and max_frames > 0")
        self.slots, self.max_frames = int(slots), int(max_frames)
        self._free = list(range(self.slots - 1, -1, -1))  # a stack: released slots are reused first
        self._used = set()
        self._lock = threading.Lock()
        self.feats = None
        if alloc:
            import torch
            self.feats = torch.empty((self.slots * self.max_frames, R.trans_input_size), dtype=torch.float32,
                                     device=device)

    @property
    def free(self):
        return len(self._free)

    def alloc(self, k):
        """Up to k free slots (fewer when the store is short)."""
        with self._lock:
            out = [self._free.pop() for _ in range(min(int(k), len(self._free)))]
            self._used.update(out)
            return out

    def release(self, slots):
        with self._lock:
            for s in slots:
                if s not in self._used:
                    raise ValueError(f"feature store slot {s} released while not in use")
                self._used.remove(s)
                self._free.append(s)

    def row(self, slot):
        return int(slot) * self.max_frames


class WavFeed:
    """The producer stage of one Server lane over WAV input (reference ServerSUT::thProducer,
    torch_sut.cpp:354-468: take up to pro_batch_size queued samples, AssembleSamples +
    AudioProcessor, enqueue each sample's features for the consumers).  Here the QSL's audio is
    resident in the lane's device HBM (GpuWavQSL, LoadSamplesToRam), the samples a producer takes
    are featurized in one launch straight into the lane's FeatureStore, and handed to the lane's
    engines.  ``ServerSUT(feeds=[...])`` runs one producer thread per feed; feeds on several
    devices (or several on one) serve one Server instance, each pulling from the shared queue only
    while its own backlog is short (``ahead``), so work goes where an engine will take it soon.

    qsl: GpuWavQSL on this lane's device; store_slots: FeatureStore size (default: ServerSUT
    sizes it to the lane's engine slots + ahead); max_frames: a store slot's rows (default the
    QSL's longest sample)."""

    def __init__(self, qsl, store_slots=None, pro_batch=512, ahead=None, max_frames=None, alloc=True, cu_mask=None):
        self.qsl, self.pro_batch, self.ahead = qsl, int(pro_batch), ahead
        self.cu_mask = cu_mask  # featurize on this CU set only (engine.cu_mask_words); None: any CU
        self._pstreams = []
        self.store_slots, self.alloc = store_slots, alloc
        self.max_frames = int(max_frames or max(int(np.max(qsl.lengths)), 1))
        self.store = None
        self.batches = 0

    @property
    def device(self):
        import torch
        return torch.device(self.qsl.device).index or 0

    def open(self, slots, ahead):
        """Sizes the lane (called by ServerSUT once engines are assigned)."""
        if self.ahead is None:
            self.ahead = int(ahead)
        if self.store is None:
            n = int(self.store_slots or slots + self.ahead)
            self.store = FeatureStore(n, self.max_frames, device=self.qsl.device, alloc=self.alloc)

    def make_stream(self):
        """The producer's stream (one per feed, kept across Server instances)."""
        if not self._pstreams:
            from .engine import PartitionedStream
            self._pstreams.append(PartitionedStream(self.device, self.cu_mask))
        return self._pstreams[0].stream

    def featurize(self, indices, slots, stream):
        """Featurize QSL samples ``indices`` into store ``slots`` (one launch), wait for it; ->
        their feature lengths (host int32)."""
        import torch
        idx = np.asarray(indices, np.int64)
        wl = self.qsl.wav_lengths[idx].astype(np.int32)
        dev = self.qsl.store.device
        with torch.cuda.device(dev), torch.cuda.stream(stream):
            off = torch.from_numpy(self.qsl.offsets[idx]).to(dev)
            wld = torch.from_numpy(wl).to(dev)
            rows = np.array([self.store.row(s) for s in slots], np.int64)
            self.qsl._featurizer().featurize_rows(self.qsl.store, wld, wl, self.store.feats, rows,
                                                  self.store.max_frames, offsets=off, stream=stream)
            stream.synchronize()
        self.batches += 1
        return self.qsl.lengths[idx]


class ServerSUT:
    """Server scenario SUT with continuous batching (reference ServerSUT, csrc/torch_sut.cpp:238-571,
    PipelineState, csrc/metadata.cpp:97-194; TorchModel::encode's split_len loop, rnnt_model.hpp:62-90).

    Each engine is one PipelineState of ``slots`` rows that carry their LSTM and greedy state from
    one round to the next.  A round (one host thread per engine, its own HIP stream):
      1. refill (PipelineState::update): free slots take waiting samples, first come first served;
         their encoder / prediction state and result row restart (the reset flags);
      2. encode one chunk of ``split_len`` frames of every busy slot from the QSL's HBM-resident
         feature store (rnnt_engine_encode_stream: per-slot offsets, h/c carried), then decode that
         chunk's frames (rnnt_engine_decode_stream: pre_g / pre_hg / pre_cg / result row carried);
      3. respond early (QuerySamplesComplete, torch_sut.cpp:542-571): every slot whose features are
         used up is answered with its token row and freed, the others continue next round.
    Encoders of the engines on one GPU take turns, so one engine's decode overlaps the next
    engine's encode.  Chunked encoding is exact (h/c carry, StackTime pairs within even chunks) and
    so is the chunked greedy decode (symbols_added / time restart at a chunk boundary exactly as
    at a frame boundary): every answer equals the Offline answer for that sample.
    QoS deferral (torch_sut.cpp:396-414): samples longer than ``qos_len`` feature frames wait until
    ``flush_queries`` (LoadGen's FlushQueries, lStop_) and then run after the regular queue.
    ``response_size`` of the reference (the minimum number of finished rows per consumer
    iteration, which amortises its CPU iteration) is subsumed: a round is one chunk and answers
    every slot that finished in it.  Latency per sample = completion - issue time.

    Inputs: ``qsl`` is a feature QSL with an HBM-resident store (GpuQSL), or {device: GpuQSL}
    replicas for engines on several GPUs.  Over WAV (the reference's processor=true Server,
    thProducer, torch_sut.cpp:354-468), pass ``feeds``: WavFeed producers, each with its own
    per-device FeatureStore; engine j is served by feed ``lanes[j]`` (default: the feeds of the
    engine's device, round-robin), the producers featurize arriving samples into their stores and
    the engines of a lane take only their lane's samples.  Latency then includes featurization."""

    def __init__(self, engines, qsl=None, slots=2048, split_len=128, qos_len=None, on_complete=None, pipelined=False,
                 feeds=None, lanes=None, engine_cu_mask=None, refill="fcfs", refill_window=2048):
        """refill: "fcfs" -- every free slot takes the oldest waiting sample (PipelineState::update);
        "tile" -- slots are refilled a 128-row tile at a time, once the whole tile is free, with the
        oldest waiting sample and the waiting ones (among the first ``refill_window``) closest to its
        length, so a tile's rows run out together and the encoder skips the tile as soon as they do
        (the tick kernel skips any done tile of a stream chunk, not only trailing ones)."""
        import threading
        from .engine import pad_batch
        if split_len <= 0 or split_len % 2:
            raise ValueError("split_len must be a positive even number of frames (StackTime pairs frames)")
        if refill not in ("fcfs", "tile"):
            raise ValueError("refill: 'fcfs' or 'tile'")
        if refill == "tile" and pipelined:
            raise ValueError("refill='tile' is implemented for the round form (pipelined=False)")
        self.refill, self.refill_window = refill, int(refill_window)
        self.engines = list(engines) if isinstance(engines, (list, tuple)) else [engines]
        self.qsl, self.split_len, self.qos_len = qsl, int(split_len), qos_len
        self.slots = pad_batch(int(slots))
        for e in self.engines:
            if e.max_batch < self.slots:
                raise ValueError(f"engine max_batch {e.max_batch} < {self.slots} slots")
        self.feeds = list(feeds) if feeds else []
        if self.feeds:
            self.lengths = np.asarray(self.feeds[0].qsl.lengths)
            if any(not np.array_equal(f.qsl.lengths, self.lengths) for f in self.feeds):
                raise ValueError("every feed must hold the same samples")
            self.lanes = self._assign_lanes(lanes)
            for f in range(len(self.feeds)):
                nl = sum(1 for x in self.lanes if x == f)
                self.feeds[f].open(nl * self.slots, self.slots)
        else:
            if qsl is None:
                raise ValueError("ServerSUT needs a feature QSL or WAV feeds")
            self._meta_qsl = next(iter(qsl.values())) if isinstance(qsl, dict) else qsl
            self.lengths = np.asarray(self._meta_qsl.lengths)
            self.lanes = [None] * len(self.engines)
        self.on_complete = on_complete
        self.pipelined = bool(pipelined)
        self.engine_cu_mask = engine_cu_mask  # engines' streams on this CU set (engine.cu_mask_words)
        self._pstreams = []
        self.responses, self.latency = {}, {}
        self._pending, self._qos = [], []  # (issue_time, QuerySample)
        self._ready = [collections.deque() for _ in self.feeds]  # per feed: (t0, sample, row, length, slot)
        self._prod_live = [False] * len(self.feeds)
        self._lane_workers = collections.Counter(x for x in self.lanes if x is not None)
        self._cv = threading.Condition()
        self._enc_locks = {}
        self._stop = self._flushed = False
        self._threads = []
        self.rounds = 0
        self.errors = []

    def warmup(self, iters=1, frames=R.MAX_FEA_LEN):
        """ServerSUT::warmup (torch_sut.cpp:328-352), before ``start``: the producers' part
        (processor=true: featurize dummy audio) and the consumers' part (dummy samples of
        MAX_FEA_LEN frames through the model) -- here every feed featurizes up to one producer batch
        of its QSL's samples into its store (slots returned afterwards) and every engine runs `iters`
        dummy samples in all its slots through the same split_len rounds its worker runs
        (encode_stream + decode_stream, reset on the first chunk, h/c and greedy state carried over
        the following chunks).  The slots' carried state is left dirty, which is harmless: a slot
        is reset whenever it takes a sample.  -> seconds spent."""
        import time
        import torch
        if self._threads:
            raise RuntimeError("ServerSUT.warmup must run before start()")
        t0 = time.perf_counter()
        for feed in self.feeds:
            k = max(1, min(feed.pro_batch, feed.store.free, len(feed.qsl.lengths)))
            slots = feed.store.alloc(k)
            try:
                st = feed.make_stream()
                feed.featurize(list(range(k)), slots, st)
                st.synchronize()
            finally:
                feed.store.release(slots)
        S, L = self.slots, self.split_len
        for eng in self.engines:
            dev = torch.device("cuda", eng.device)
            with torch.cuda.device(eng.device):
                st = self._new_stream(eng.device)
                g = torch.Generator(device=dev)
                g.manual_seed(0)
                store = torch.randn((int(frames), R.trans_input_size), device=dev, generator=g)  # one dummy sample
                res = torch.empty((S, eng.max_res), dtype=torch.int32, device=dev)
                rl = torch.zeros(S, dtype=torch.int32, device=dev)
                with torch.cuda.stream(st):
                    for _ in range(int(iters)):
                        for c0 in range(0, int(frames), L):
                            cl = min(L, int(frames) - c0)
                            lens_h = np.full(S, cl, np.int32)
                            d_reset = torch.full((S,), 1 if c0 == 0 else 0, dtype=torch.int32, device=dev)
                            d_lens = torch.from_numpy(lens_h).to(dev)
                            d_off = torch.full((S,), c0, dtype=torch.int64, device=dev)
                            eng.encode_stream(store, d_off, d_lens, lens_h, d_reset, cl, S, S, stream=st)
                            eng.decode_stream(res, rl, d_reset, stream=st)
                    st.synchronize()
                del store, res, rl
        _release_cached(self.engines)
        return time.perf_counter() - t0

    def _assign_lanes(self, lanes):
        if lanes is not None:
            lanes = [int(x) for x in lanes]
            if len(lanes) != len(self.engines) or any(not 0 <= x < len(self.feeds) for x in lanes):
                raise ValueError("lanes: one feed index per engine")
        else:
            lanes, turn = [], collections.Counter()
            for e in self.engines:
                mine = [f for f, fd in enumerate(self.feeds) if fd.device == e.device]
                if not mine:
                    raise ValueError(f"no WAV feed on device {e.device}")
                lanes.append(mine[turn[e.device] % len(mine)])
                turn[e.device] += 1
        for e, f in zip(self.engines, lanes):
            if self.feeds[f].device != e.device:
                raise ValueError(f"engine on device {e.device} assigned to a feed on device {self.feeds[f].device}")
        if set(lanes) != set(range(len(self.feeds))):
            raise ValueError("every feed needs at least one engine")
        return lanes

    def _new_stream(self, device):
        import torch
        if self.engine_cu_mask is None:
            return torch.cuda.Stream(device=torch.device("cuda", device))
        from .engine import PartitionedStream
        ps = PartitionedStream(device, self.engine_cu_mask)
        self._pstreams.append(ps)
        return ps.stream

    def _store_for(self, j):
        """(feature store tensor, lane) of engine j."""
        f = self.lanes[j]
        if f is not None:
            return self.feeds[f].store.feats, f
        q = self.qsl[self.engines[j].device] if isinstance(self.qsl, dict) else self.qsl
        return q.feats, None

    # LoadGen-facing surface -------------------------------------------------------------
    def start(self):
        import threading
        for e in self.engines:
            self._enc_locks.setdefault(e.device, threading.Lock())
        self._start_producers()
        for j in range(len(self.engines)):
            t = threading.Thread(target=self._worker_pl if self.pipelined else self._worker, args=(j,), daemon=True)
            t.start()
            self._threads.append(t)

    def _start_producers(self):
        import threading
        for f in range(len(self.feeds)):
            self._prod_live[f] = True
            t = threading.Thread(target=self._producer, args=(f,), daemon=True)
            t.start()
            self._threads.append(t)

    def issue_query(self, samples, now=None):
        import time
        now = time.perf_counter() if now is None else now
        with self._cv:
            for s in samples:
                long_ = self.qos_len is not None and int(self.lengths[s.index]) > self.qos_len
                (self._qos if long_ else self._pending).append((now, s))
            self._cv.notify_all()

    def flush_queries(self):
        """LoadGen's FlushQueries (torch_sut.hpp:120-122): no more queries; deferred QoS samples run."""
        with self._cv:
            self._flushed = True
            self._cv.notify_all()

    def stop(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        for t in self._threads:
            t.join()
        for ps in self._pstreams:
            ps.close()
        self._pstreams = []

    # producers (WAV feeds) ------------------------------------------------------------------
    def _source(self):
        """The queue samples are taken from now: regular first, deferred QoS samples once issuing
        stopped (torch_sut.cpp:408-414); None when both are empty / held."""
        if self._pending:
            return self._pending
        if self._flushed and self._qos:
            return self._qos
        return None

    def _producer(self, f):
        """thProducer (torch_sut.cpp:354-468) of feed f: while the lane's backlog of featurized,
        not yet taken samples is under ``ahead`` and its store has room, take up to pro_batch
        queued samples (a burst is split over the feeds), featurize them into the store in one
        launch and hand them to the lane's engines."""
        feed = self.feeds[f]
        store, ready = feed.store, self._ready[f]
        try:
            st = feed.make_stream()
            while True:
                with self._cv:
                    while True:
                        if self._lane_workers[f] <= 0:  # the lane's engines failed
                            return
                        src = self._source()
                        room = min(store.free, feed.ahead - len(ready))
                        if src and room > 0:
                            share = -(-len(src) // len(self.feeds))
                            k = max(1, min(room, feed.pro_batch, share))
                            items = src[:k]
                            del src[:k]
                            break
                        if self._stop and src is None:
                            return
                        self._cv.wait()
                slots = store.alloc(len(items))  # only this thread allocates: room >= len(items)
                try:
                    lens = feed.featurize([s.index for _, s in items], slots, st)
                except Exception as ex:  # surface in the caller, never hang the query
                    store.release(slots)
                    self.errors.append(ex)
                    for t0, s in items:
                        self.latency[s.id] = float("inf")
                    continue
                with self._cv:
                    ready.extend((t0, s, store.row(sl), int(L), sl) for (t0, s), sl, L in zip(items, slots, lens))
                    self._cv.notify_all()
        except Exception as ex:
            self.errors.append(ex)
        finally:
            with self._cv:
                self._prod_live[f] = False
                self._cv.notify_all()

    def _release(self, lane, slots):
        """Store slots whose samples are fully encoded go back to the lane's producer."""
        if lane is None or not len(slots):
            return
        self.feeds[lane].store.release(slots)
        with self._cv:
            self._cv.notify_all()

    # consumer -----------------------------------------------------------------------------
    def _grouped(self, n_items, k, length_of):
        """Indices (into a waiting list of n_items) of up to k samples taken in groups of TILE: each
        group is the oldest sample not yet taken and the ones closest to its length among the first
        refill_window samples not yet taken, in arrival order within the group."""
        w = min(n_items, self.refill_window + k)
        if w == 0 or k <= 0:
            return []
        L = np.fromiter((length_of(i) for i in range(w)), np.int64, w)
        taken = np.zeros(w, bool)
        out = []
        while len(out) < k and not taken.all():
            elig = np.flatnonzero(~taken)[: self.refill_window]  # the window slides past taken samples
            head = int(elig[0])
            d = np.abs(L[elig] - L[head]).astype(np.float64) + np.arange(len(elig)) * 1e-9  # ties: older first
            m = min(self.TILE, k - len(out), len(elig))
            pick = np.sort(elig[np.argpartition(d, m - 1)[:m]])
            taken[pick] = True
            out.extend(int(i) for i in pick)
        return out

    TILE = 128  # the tick kernel's batch-row tile (ENC_ROW_TILE)

    def _take(self, k, busy, lane=None):
        """Up to k samples for free slots, as (issue_time, QuerySample, first store row, frames,
        store slot or None); blocks only while this engine has no busy slot.  With feeds: the
        lane's featurized samples.  None: stopped and nothing left for this engine.  With
        refill='tile' the samples come in groups of TILE similar lengths (``_grouped``)."""
        with self._cv:
            while True:
                if lane is not None:
                    rd = self._ready[lane]
                    if rd and k > 0:
                        if self.refill == "tile":
                            w = min(len(rd), self.refill_window + k)
                            items = [rd.popleft() for _ in range(w)]  # only the window can be taken from
                            idx = self._grouped(len(items), k, lambda i: items[i][3])
                            keep = set(idx)
                            out = [items[i] for i in idx]
                            rd.extendleft(reversed([x for i, x in enumerate(items) if i not in keep]))
                        else:
                            out = [rd.popleft() for _ in range(min(k, len(rd)))]
                        self._cv.notify_all()  # the producer may have room again
                        return out
                    if busy or k == 0:
                        return []
                    if self._stop and not self._prod_live[lane]:
                        return None
                else:
                    src = self._source()
                    if src and k > 0:
                        if self.refill == "tile":
                            idx = self._grouped(len(src), k, lambda i: self.lengths[src[i][1].index])
                            keep = set(idx)
                            out = [src[i] for i in idx]
                            w = max(idx) + 1  # only the window can be taken from: rebuild just that prefix
                            src[:w] = [x for i, x in enumerate(src[:w]) if i not in keep]
                        else:
                            out = src[:k]
                            del src[:k]
                        q = self._meta_qsl  # replicas share offsets / lengths
                        return [(t0, s, int(q.offsets[s.index]), int(q.lengths[s.index]), None) for t0, s in out]
                    if busy or k == 0:
                        return []
                    if self._stop:
                        return None
                self._cv.wait()

    def _worker(self, j):
        import time
        import torch
        eng = self.engines[j]
        S, L = self.slots, self.split_len
        dev = torch.device("cuda", eng.device)
        with torch.cuda.device(eng.device):
            st = self._new_stream(eng.device)
            res = torch.empty((S, eng.max_res), dtype=torch.int32, device=dev)
            rl = torch.zeros(S, dtype=torch.int32, device=dev)
            # per-round host -> device inputs: reset flags, chunk lengths, row offsets (pinned)
            h_reset = torch.zeros(S, dtype=torch.int32).pin_memory()
            h_lens = torch.zeros(S, dtype=torch.int32).pin_memory()
            h_off = torch.zeros(S, dtype=torch.int64).pin_memory()
            d_reset = torch.zeros(S, dtype=torch.int32, device=dev)
            d_lens = torch.zeros(S, dtype=torch.int32, device=dev)
            d_off = torch.zeros(S, dtype=torch.int64, device=dev)
        store, lane = self._store_for(j)
        sample = [None] * S               # (issue_time, QuerySample) per slot
        pos = np.zeros(S, np.int64)       # next frame of the slot's sample
        remain = np.zeros(S, np.int32)    # frames left
        base = np.zeros(S, np.int64)      # first stored row of the slot's sample
        sslot = [None] * S                # the sample's feature store slot (WAV feeds)
        try:
            while True:
                free = [i for i in range(S) if sample[i] is None]
                if self.refill == "tile":  # whole free tiles, filled group by group
                    TL = self.TILE
                    ftiles = [t for t in range(S // TL) if all(sample[i] is None for i in range(t * TL, (t + 1) * TL))]
                    new = self._take(len(ftiles) * TL, busy=len(free) < S, lane=lane)
                    free = [t * TL + j for t in ftiles for j in range(TL)]
                else:
                    new = self._take(len(free), busy=len(free) < S, lane=lane)
                if new is None:
                    return
                rs = h_reset.numpy()
                rs[:] = 0
                for i, (t0, smp, row, nfr, sl) in zip(free, new):
                    sample[i], sslot[i] = (t0, smp), sl
                    pos[i], remain[i], base[i] = 0, nfr, row
                    rs[i] = 1
                busy = np.array([x is not None for x in sample])
                if not busy.any():
                    continue
                cl = np.where(busy, np.minimum(remain, L), 0).astype(np.int32)
                h_lens.numpy()[:] = cl
                h_off.numpy()[:] = np.where(busy, base + pos, 0)
                T = max(int(cl.max()), 1)
                with torch.cuda.device(eng.device), torch.cuda.stream(st):
                    d_reset.copy_(h_reset, non_blocking=True)
                    d_lens.copy_(h_lens, non_blocking=True)
                    d_off.copy_(h_off, non_blocking=True)
                    with self._enc_locks[eng.device]:  # encoders on one GPU take turns
                        eng.encode_stream(store, d_off, d_lens, cl, d_reset, T, S, S, stream=st)
                        st.synchronize()
                    pos += cl
                    remain -= cl
                    done = np.nonzero(busy & (remain == 0))[0]
                    rel = [sslot[i] for i in done]
                    for i in done:
                        sslot[i] = None
                    self._release(lane, rel)  # their features are read
                    eng.decode_stream(res, rl, d_reset, stream=st)
                    if len(done):
                        di = torch.from_numpy(done).to(dev)
                        lens_d = rl.index_select(0, di)
                        rlh = lens_d.cpu().numpy()
                        toks = res.index_select(0, di)[:, : max(1, int(rlh.max()))].cpu().numpy()
                    else:
                        st.synchronize()
                self.rounds += 1
                now = time.perf_counter()
                for k, i in enumerate(done):
                    t0, s = sample[i]
                    row = toks[k, : rlh[k]].copy()
                    self.responses[s.id] = row
                    self.latency[s.id] = now - t0
                    if self.on_complete:
                        self.on_complete(s, row)
                    sample[i] = None
        except Exception as ex:  # surface in the caller, never hang the query
            self.errors.append(ex)
            for item in sample:
                if item is not None:
                    self.latency[item[1].id] = float("inf")
            self._fail_worker(lane, sslot)

    def _fail_worker(self, lane, held):
        """A failed engine: its store slots go back; when it was its lane's last engine, what is
        queued for the lane is answered (latency inf) and the lane's producer stops taking work,
        so the query still ends."""
        if lane is None:
            return
        self._release(lane, [sl for sl in held if sl is not None])
        with self._cv:
            self._lane_workers[lane] -= 1
            if self._lane_workers[lane] <= 0:
                rd = self._ready[lane]
                while rd:
                    t0, s, _, _, sl = rd.popleft()
                    self.latency[s.id] = float("inf")
                    self.feeds[lane].store.release([sl])
            self._cv.notify_all()


    def _worker_pl(self, j):
        """Pipelined rounds (``pipelined=True``): this thread plans and encodes round k+1 while a
        decode thread of the same engine decodes round k (rnnt_engine_encode_stream_pl /
        decode_stream_pl).  Planning needs only the host frame counters, so a slot whose features
        run out in round k is refilled in round k+1 before round k's decode has answered it; the
        decode thread reads finished rows back before it starts round k+1's decode, which resets
        them.  Answers are those of ``_worker``."""
        import queue
        import threading
        import time
        import torch
        eng = self.engines[j]
        S, L = self.slots, self.split_len
        dev = torch.device("cuda", eng.device)
        NR = 4  # reset-flag ring: round k's flags live until its decode completed (k+3 reuses them)
        with torch.cuda.device(eng.device):
            est, dst = self._new_stream(eng.device), self._new_stream(eng.device)
            res = torch.empty((S, eng.max_res), dtype=torch.int32, device=dev)
            rl = torch.zeros(S, dtype=torch.int32, device=dev)
            h_reset = torch.zeros(S, dtype=torch.int32).pin_memory()
            h_lens = torch.zeros(S, dtype=torch.int32).pin_memory()
            h_off = torch.zeros(S, dtype=torch.int64).pin_memory()
            d_reset = [torch.zeros(S, dtype=torch.int32, device=dev) for _ in range(NR)]
            d_lens = torch.zeros(S, dtype=torch.int32, device=dev)
            d_off = torch.zeros(S, dtype=torch.int64, device=dev)
        store, lane = self._store_for(j)
        sample = [None] * S
        pos = np.zeros(S, np.int64)
        remain = np.zeros(S, np.int32)
        base = np.zeros(S, np.int64)
        sslot = [None] * S
        rounds = queue.Queue(maxsize=2)  # (reset ring index, [(slot, (issue_time, QuerySample))])
        started = [0]  # rounds whose decode has been called
        scv = threading.Condition()

        def decoder():
            failed = False
            while True:
                item = rounds.get()
                with scv:
                    started[0] += 1
                    scv.notify()
                if item is None:
                    return
                r, done = item
                try:  # keep decoding after a failure: the encode side waits for each hand-off
                    with torch.cuda.device(eng.device), torch.cuda.stream(dst):
                        eng.decode_stream_pl(res, rl, d_reset[r], stream=dst)
                        if done and not failed:
                            di = torch.tensor([i for i, _ in done], device=dev)
                            rlh = rl.index_select(0, di).cpu().numpy()
                            toks = res.index_select(0, di)[:, : max(1, int(rlh.max()))].cpu().numpy()
                        else:
                            dst.synchronize()
                    if failed:
                        raise RuntimeError("an earlier pipelined decode failed")
                    now = time.perf_counter()
                    for k, (_, (t0, smp)) in enumerate(done):
                        row = toks[k, : rlh[k]].copy()
                        self.responses[smp.id] = row
                        self.latency[smp.id] = now - t0
                        if self.on_complete:
                            self.on_complete(smp, row)
                    self.rounds += 1
                except Exception as ex:
                    if not failed:
                        self.errors.append(ex)
                    failed = True
                    for _, (_, smp) in done:
                        self.latency[smp.id] = float("inf")

        dthread = threading.Thread(target=decoder, daemon=True)
        dthread.start()
        k = 0
        try:
            while True:
                free = [i for i in range(S) if sample[i] is None]
                if self.refill == "tile":  # whole free tiles, filled group by group
                    TL = self.TILE
                    ftiles = [t for t in range(S // TL) if all(sample[i] is None for i in range(t * TL, (t + 1) * TL))]
                    new = self._take(len(ftiles) * TL, busy=len(free) < S, lane=lane)
                    free = [t * TL + j for t in ftiles for j in range(TL)]
                else:
                    new = self._take(len(free), busy=len(free) < S, lane=lane)
                if new is None:
                    return
                rs = h_reset.numpy()
                rs[:] = 0
                for i, (t0, smp, row, nfr, sl) in zip(free, new):
                    sample[i], sslot[i] = (t0, smp), sl
                    pos[i], remain[i], base[i] = 0, nfr, row
                    rs[i] = 1
                busy = np.array([x is not None for x in sample])
                if not busy.any():
                    continue
                cl = np.where(busy, np.minimum(remain, L), 0).astype(np.int32)
                h_lens.numpy()[:] = cl
                h_off.numpy()[:] = np.where(busy, base + pos, 0)
                T = max(int(cl.max()), 1)
                r = k % NR
                with scv:  # round k's encode hands over once round k-1's decode began: wait for
                    while started[0] < k:  # that outside the encoders' turn
                        scv.wait()
                with torch.cuda.device(eng.device), torch.cuda.stream(est):
                    d_reset[r].copy_(h_reset, non_blocking=True)
                    d_lens.copy_(h_lens, non_blocking=True)
                    d_off.copy_(h_off, non_blocking=True)
                    with self._enc_locks[eng.device]:  # encoders on one GPU take turns
                        eng.encode_stream_pl(store, d_off, d_lens, cl, d_reset[r], T, S, S, stream=est)
                        est.synchronize()
                pos += cl
                remain -= cl
                done = [(int(i), sample[i]) for i in np.nonzero(busy & (remain == 0))[0]]
                rel = [sslot[i] for i, _ in done]
                for i, _ in done:
                    sample[i], sslot[i] = None, None
                self._release(lane, rel)  # their features are read
                rounds.put((r, done))
                k += 1
        except Exception as ex:  # surface in the caller, never hang the query
            self.errors.append(ex)
            for item in sample:
                if item is not None:
                    self.latency[item[1].id] = float("inf")
            self._fail_worker(lane, sslot)
        finally:
            rounds.put(None)
            dthread.join()


class DynamicBatchServerSUT:
    """Server scenario SUT by dynamic batching of whole utterances: one worker thread per engine
    (HIP stream each); whenever a worker is free it takes every pending sample (up to max_batch,
    longest first), assembles the batch on the device (any QSL, incl. the WAV featurizer path),
    encodes (encoders take turns), decodes and completes each sample with its token row.
    ``ServerSUT`` (continuous batching with carried state) is the reference's structure; this one
    serves QSLs without a resident feature store.  Latency per sample = completion - issue time."""

    def __init__(self, engines, qsl, max_batch=2048, on_complete=None):
        import threading
        self.engines = list(engines) if isinstance(engines, (list, tuple)) else [engines]
        self.qsl, self.max_batch = qsl, max_batch
        self.on_complete = on_complete
        self.responses, self.latency = {}, {}
        self._pending = []  # (issue_time, QuerySample)
        self._cv = threading.Condition()
        self._enc_lock = threading.Lock()
        self._stop = False
        self._threads = []
        self.batches = 0
        self.batch_log = []  # (engine index, sample ids in batch row order) per batch, for diagnostics
        self.errors = []

    def start(self):
        import threading
        for j in range(len(self.engines)):
            t = threading.Thread(target=self._worker, args=(j,), daemon=True)
            t.start()
            self._threads.append(t)

    def issue_query(self, samples, now=None):
        import time
        now = time.perf_counter() if now is None else now
        with self._cv:
            self._pending.extend((now, s) for s in samples)
            self._cv.notify()

    def stop(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        for t in self._threads:
            t.join()

    def _take(self):
        with self._cv:
            while not self._pending and not self._stop:
                self._cv.wait()
            if not self._pending:
                return None
            batch = self._pending[: self.max_batch]
            del self._pending[: self.max_batch]
            return batch

    def _worker(self, j):
        import time
        import torch
        eng = self.engines[j]
        st = torch.cuda.Stream()
        while True:
            batch = self._take()
            if batch is None:
                return
            try:
                batch.sort(key=lambda b: -int(self.qsl.lengths[b[1].index]))  # rnnt_qsl.cpp:104-133
                n = len(batch)
                self.batch_log.append((j, [s.id for _, s in batch]))
                with torch.cuda.stream(st):
                    x, lens, bl = self.qsl.assemble([b[1].index for b in batch])
                    res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
                    rl = torch.empty(n, dtype=torch.int32, device="cuda")
                with self._enc_lock:
                    eng.encode(x, lens, bl, n=n, stream=st)
                    st.synchronize()
                eng.decode(res, rl, stream=st)
                with torch.cuda.stream(st):
                    rlh = rl.cpu()
                    toks = res[:, : max(1, int(rlh.max()))].cpu().numpy()
                done = time.perf_counter()
                rlh = rlh.numpy()
                for i, (t0, s) in enumerate(batch):
                    row = toks[i, : rlh[i]].copy()
                    self.responses[s.id] = row
                    self.latency[s.id] = done - t0
                    if self.on_complete:
                        self.on_complete(s, row)
                self.batches += 1
            except Exception as ex:  # surface in the caller, never hang the query
                self.errors.append(ex)
                for t0, s in batch:
                    self.latency[s.id] = float("inf")
