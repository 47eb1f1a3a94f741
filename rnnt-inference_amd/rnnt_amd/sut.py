"""Query Sample Library and Offline SUT over the HIP engine.

Mirrors the reference's LoadGen-facing surface (the real MLPerf LoadGen is not installable
offline, so the query / response types are plain Python):
  * ``RNNTQSL``   csrc/rnnt_qsl.{hpp,cpp} / models/rnnt_qsl.py: holds per-sample features
                  [T_i, 240] and lengths; ``sort`` is the length-descending bucket sort
                  (rnnt_qsl.cpp:104-133); ``assemble`` pads a batch to [T_max, n_pad, 256]
                  (AssembleSamples, rnnt_qsl.cpp:150-188).
  * ``OfflineSUT`` csrc/torch_sut.cpp:88-236 / models/pytorch_sut.py:58-118: issue_queries
                  sorts, takes <= batch_size samples per batch, runs encode+decode on its GPU
                  and completes each sample with its int32 token row (res_len*4 bytes,
                  QuerySamplesComplete, torch_sut.cpp:221-236).
Multi-GPU: one process per GPU, each with its own engine(s); a query's sorted samples are
dealt to ranks in batch-sized chunks (snake order, so every rank gets the same length mix).
There is no data-path collective: results are completed per rank.  Within a GPU, several
engines (each with its own HIP stream and host thread, like the reference's INTER worker
threads, torch_sut.cpp:143-182) keep batches in flight; encoders take turns so one batch's
latency-bound greedy decode overlaps the next batch's encoder.
"""
from dataclasses import dataclass

import numpy as np

from .config import RNNTParam as R
from .engine import pad_batch


@dataclass
class QuerySample:
    id: int
    index: int


class RNNTQSL:
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

    def __len__(self):
        return self.count

    def sort(self, samples, reverse=True):
        """Bucket sort by feature length, longest first (rnnt_qsl.cpp:104-133)."""
        lmin, lmax = int(self.lengths.min()), int(self.lengths.max())
        buckets = [[] for _ in range(lmax - lmin + 1)]
        for s in samples:
            L = int(self.lengths[s.index])
            buckets[(lmax - L) if reverse else (L - lmin)].append(s)
        return [s for b in buckets for s in b]

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


def deal_batches(sorted_samples, batch_size, rank=0, world=1):
    """Split a length-sorted query into batch_size chunks and deal them to ranks in snake
    order (0,1,..,w-1,w-1,..,0,0,..) so every rank gets a similar share of long and short
    utterances; returns this rank's chunks."""
    chunks = [sorted_samples[i:i + batch_size] for i in range(0, len(sorted_samples), batch_size)]
    mine = []
    for i, ch in enumerate(chunks):
        r = i % world if (i // world) % 2 == 0 else world - 1 - (i % world)
        if r == rank:
            mine.append(ch)
    return mine


class OfflineSUT:
    def __init__(self, engine, qsl, batch_size=1024, rank=0, world=1, on_complete=None):
        """engine: one Engine, or a list of Engines on this GPU (one batch in flight each)."""
        self.engines = list(engine) if isinstance(engine, (list, tuple)) else [engine]
        self.engine = self.engines[0]
        self.qsl, self.batch_size = qsl, batch_size
        self.rank, self.world = rank, world
        self.on_complete = on_complete
        self.responses = {}

    def issue_queries(self, samples):
        import threading
        import torch
        batches = deal_batches(self.qsl.sort(samples), self.batch_size, self.rank, self.world)
        k = len(self.engines)
        streams = [torch.cuda.Stream() for _ in range(k)] if k > 1 else [torch.cuda.current_stream()]
        done = [None] * len(batches)
        enc_lock = threading.Lock()

        def worker(j):
            eng, st = self.engines[j], streams[j]
            for bi in range(j, len(batches), k):
                batch = batches[bi]
                x, lens = self.qsl.assemble([s.index for s in batch])
                n = len(batch)
                with torch.cuda.stream(st):
                    xd = torch.from_numpy(x).cuda()
                    ld = torch.from_numpy(lens).cuda()
                    res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
                    rl = torch.empty(n, dtype=torch.int32, device="cuda")
                with enc_lock:
                    eng.encode(xd, ld, lens[:n], n=n, stream=st)
                    st.synchronize()
                eng.decode(res, rl, stream=st)
                done[bi] = (batch, res, rl, xd, ld)

        if k == 1:
            worker(0)
        else:
            ths = [threading.Thread(target=worker, args=(j,)) for j in range(k)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        for st in streams:
            st.synchronize()
        for batch, res, rl, _, _ in done:
            self.query_samples_complete(batch, res, rl)

    def query_samples_complete(self, batch, res, res_len):
        """Response = int32 tokens [res_len] per sample (torch_sut.cpp:221-236)."""
        rl = res_len.cpu().numpy()
        width = int(rl.max()) if len(rl) else 0
        toks = res[:, :max(width, 1)].cpu().numpy()
        for i, s in enumerate(batch):
            row = toks[i, : rl[i]].copy()
            self.responses[s.id] = row
            if self.on_complete:
                self.on_complete(s, row)

    def flush_queries(self):
        pass


class GpuQSL:
    """QSL with every sample's features resident in HBM, ragged ([sum T_i, 240] fp32), and the
    AssembleSamples gather done on the device (LoadSamplesToRam + AssembleSamples,
    rnnt_qsl.cpp:150-188).  Synthetic N(0,1) features, seeded."""

    def __init__(self, lengths, seed, device="cuda"):
        import torch
        self.lengths = np.asarray(lengths, np.int32)
        self.count = len(self.lengths)
        self.offsets = np.concatenate([[0], np.cumsum(self.lengths)[:-1]]).astype(np.int64)
        g = torch.Generator(device=device)
        g.manual_seed(int(seed))
        self.feats = torch.randn((int(self.lengths.sum()), R.trans_input_size), device=device, generator=g)
        self.device = device

    def __len__(self):
        return self.count

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


class GpuWavQSL:
    """WAV=true QSL (launch_sut.sh:53-55; AssembleSamples(processor=true) + AudioProcessor,
    rnnt_qsl.cpp:150-188, torch_sut.cpp:192-200): every sample's 16 kHz audio resident in HBM,
    ragged, and ``assemble`` runs the GPU featurizer straight from that storage (per-row
    offsets: no padded [N, max_len] copy) into the engine's [T, n_pad, 256] layout.  One
    featurizer per calling thread (its workspace is per object), on the caller's stream.
    ``lengths`` are the feature lengths (what the SUT sorts by), ``wav_lengths`` the samples."""

    def __init__(self, wavs, device="cuda", featurizer_kwargs=None):
        import threading
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

    def __len__(self):
        return self.count

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


class ServerSUT:
    """Server scenario SUT (reference ServerSUT, csrc/torch_sut.cpp:238-571, with
    PipelineState continuous batching, metadata.cpp:97-194).  MI355X form: one worker thread
    per engine (HIP stream each); whenever a worker is free it takes every pending sample (up
    to max_batch, longest first), assembles the batch on the device, encodes (encoders take
    turns), decodes and completes each sample with its token row.  A batch's latency on the GPU
    (tens of ms) is far below the 1 s Server budget, so dynamic batching replaces the
    reference's slot refilling.  Latency per sample = completion - issue time."""

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
