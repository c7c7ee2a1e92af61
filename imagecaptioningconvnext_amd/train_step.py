"""Fused teacher-forced train step (train.py:240-302, trainMultiGPU.py:339-420) on HIP + RCCL.

Per step, exactly the reference's work:
  encoder(imgs) in train mode (frozen weights, stochastic depth active)      train.py:242,261
  decoder teacher-forced forward + packed CE (+ alpha reg for LSTM)          :262-276
  zero_grad + backward (into the fine-tuned encoder children too, if any)     :278-281
  DDP gradient averaging (bucketed RCCL all-reduces of the flat grad buffer)  trainMultiGPU.py:233,384
  clip_gradient (clamp +-5) + Adam step (one fused kernel per optimizer)      :284-291 / :387-394
  loss/token/top-5 metrics (reduceLossAndTokens + accuracy all-reduces,
  fused into one 3-float all-reduce; read back lazily, no per-step host sync) :396-403

With ``graph=True`` the encoder + decoder forward/backward (several hundred kernel launches,
most of them small on the LSTM recurrence) is captured once into a HIP graph and replayed
per step; the batch is copied into the graph's static input buffers first.

Data parallel (world > 1): the gradient all-reduce is bucketed like DDP's.  The engines name
their buckets in backward order (LSTM: embedding + fc, 64 % of its parameters, final before the
weight-gradient GEMMs of the rest; Transformer: one per decoder layer, last layer first, or one
for all layers in the pipelined schedule; fine-tuned encoder: the decoder rest, then ~25 MiB
encoder buckets).  Each bucket's RCCL all-reduce runs on a communication stream while the rest of
the backward runs (eager: issued from the backward's hook; graph mode: the step is captured as
one graph per hook + 1 and each bucket is reduced between two replays).  What no bucket covers
is reduced after the backward, then clip + Adam (trainMultiGPU.py:384-394).  Dropout and
stochastic-depth masks stay fresh per replay through the device step counter
(imgcap_set_seed_counter) bumped inside the graph.  The all-reduce and the Adam step (whose
bias correction depends on the host step count) run eagerly after the replay.
"""
import os

import torch
import torch.distributed as dist

from . import kernels as K


# two-branch graph: where the encoder branch forks off the decoder stream -- at the start of the
# step ("start") or after the decoder forward ("bwd": the encoder overlaps the backward only).
# Measured (bench, 1x MI355X, two runs each): C2 8,254 vs 8,366 img/s (within spread), C3 16,605
# vs 15,108, C4 7,007 vs 6,117 -- "start" stays the default.
PIPE_FORK = os.environ.get("IMGCAP_PIPE_FORK", "start")


def _trainable(encoder):
    """Encoder with fine-tuned children (any module exposing the Encoder surface)."""
    fn = getattr(encoder, "trainable", None)
    return bool(fn()) if callable(fn) else False


def _complement(ranges, n):
    """[lo, hi) pieces of [0, n) that no range in ``ranges`` covers (ranges disjoint)."""
    out, at = [], 0
    for lo, hi in sorted(ranges):
        if lo > at:
            out.append((at, lo))
        at = max(at, hi)
    if at < n:
        out.append((at, n))
    return out


def _abandon_capture(g, streams):
    """A call failed inside a capture: join the forked streams and end the capture, so the
    exception reaches the caller instead of the graph's destructor aborting the process (a
    CUDAGraph destroyed while its stream still captures)."""
    cur = torch.cuda.current_stream()
    for st in streams:
        try:
            cur.wait_stream(st)
        except Exception:  # noqa: BLE001 -- best effort; the original error is re-raised
            pass
    K._open_forks.clear()
    try:
        g.capture_end()
    except Exception:  # noqa: BLE001
        pass


class _SeqGraphs:
    """The sequential-schedule step as two captured graphs (encoder half, decoder half)."""

    def __init__(self, enc, dec):
        self.enc, self.dec = enc, dec


class TeacherForcedTrainer:
    def __init__(self, encoder, decoder, *, lstm, decoder_lr=1e-4, encoder_lr=1e-4, grad_clip=5.0, alphaC=1.0,
                 pad_id=0, process_group=None, graph=False, pipeline=False, len_buckets=True, collectives="auto"):
        self.encoder = encoder
        self.decoder = decoder
        self.lstm = lstm
        self.decoder_lr = decoder_lr
        self.encoder_lr = encoder_lr
        self.grad_clip = grad_clip
        self.alphaC = alphaC
        self.pad_id = pad_id
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        # the DDP path (buckets, hooks, split graphs, the comm stream, the metric all-reduce): with
        # more than one rank ("auto"), or "always" -- one rank of an initialised process group going
        # through every collective of the step (tests: a 1-rank RCCL group executes the same
        # schedule the 8-rank node does, bitwise the no-collective step)
        if collectives not in ("auto", "always"):
            raise ValueError("collectives: 'auto' or 'always'")
        if collectives == "always" and not (dist.is_available() and dist.is_initialized()):
            raise ValueError("collectives='always' needs an initialised process group")
        self.ddp = self.world > 1 or collectives == "always"
        self.eng = decoder.engine()
        self._metric_log = []
        # LSTM length buckets (decoder.py:91,100-111: steps t >= a caption's decode length do no
        # work): a batch whose longest caption is known on the host (CPU caplens, or step()'s
        # max_caplen) runs T = the next multiple of 8 >= its longest decode length instead of
        # L - 1 -- the vocab projection, CE, dlogits, weight-gradient GEMMs and every per-step
        # buffer shrink with it.  One captured graph set per bucket; None = L - 1.
        # Transformer: the same buckets over positions -- L' = the next multiple of 8 >= the longest
        # caption (positions past every caption are key-padding-masked and carry no loss rows, so
        # the first L' positions train exactly what L positions do; transformerDecoder.py:88-108)
        self.len_buckets = bool(len_buckets)
        self._cur_T = None
        self._seq_T = None
        self._seq_store = {}
        self.graph = graph
        self._graph = None
        # pipeline: the frozen encoder's forward of batch i runs on a second stream beside the
        # decoder forward/backward of batch i-1 (the LSTM recurrence leaves most CUs idle);
        # step(i) returns the metrics of batch i-1 and flush() finishes the last batch.  The
        # parameter updates are exactly the sequential ones (the encoder is frozen).
        self.pipeline = pipeline
        self._pipe = None
        if lstm and not os.environ.get("IMGCAP_LSTM_GROUPS"):
            # LSTM recurrences as two row groups in their one launch (lstm_persist.hip,
            # split_rows): beside the pipelined encoder branch only the forward is split (the
            # encoder needs the CUs the backward would take); the sequential schedule splits both
            self.eng.row_groups = 4 | (1 if pipeline else 3)
        # bucketed gradient all-reduce (world > 1): self._buckets = [(FlatParams, [(lo, hi), ..]),
        # ..] in the order the engines' backward passes call the bucket hook; each is reduced on
        # self._comm as soon as its gradients are final, while the rest of the backward runs
        self._feat_slot = None   # sequential graph: encoder features between the two graphs
        self._feat_meta = None
        self._enc_saved = None
        self._buckets = None
        self._hook_mode = None   # None | "eager" (issue the bucket now) | "split" (capture split)
        self._split = None
        self._next_bucket = 0    # hook calls so far in the step being run / captured
        self._issued = 0         # buckets already in flight when _update runs
        self._comm = None
        if self.ddp and torch.cuda.is_available() and self.eng.fp.grad.is_cuda:
            self._comm = torch.cuda.Stream(device=self.eng.fp.grad.device)
        if self.ddp:
            # DDP construction broadcasts rank 0's parameters (trainMultiGPU.py:233); the encoder is
            # broadcast too because its weights are randomly initialised here (SURVEY.md §7 v)
            dist.broadcast(self.eng.fp.flat, 0, group=process_group)
            self.eng.fp.refresh_shadow()
            for p in encoder.parameters():
                dist.broadcast(p.data, 0, group=process_group)
        # fine-tuned encoder children (Encoder.fine_tune, train.py:113-114): their own flat
        # parameter/grad/Adam buffers, trained with encoder_lr after the same all-reduce
        self.enc_eng = encoder.engine() if _trainable(encoder) else None
        self._plan_buckets()

    def _plan_buckets(self):
        """DDP gradient buckets (trainMultiGPU.py:233-235,256,384: torch DDP all-reduces ~25 MiB
        buckets as the backward produces them): the decoder engine's (LSTM: embedding + fc;
        Transformer: one per layer), then, with a fine-tuned encoder, the rest of the decoder
        (final before the encoder backward starts) and the encoder's ~25 MiB buckets.  What no
        bucket covers is reduced in _update.  Every element is summed once either way, so the
        averaged gradients are the same as one all-reduce of each flat buffer."""
        self._buckets = None
        if not self.ddp or not hasattr(self.eng, "grad_buckets"):
            return
        if hasattr(self.eng, "merged_layer_bucket"):
            # pipelined frozen-encoder schedule: the next batch's encoder branch joins the captured
            # step at its first split, so per-layer buckets (the first right after the last layer's
            # backward) would put the encoder in series with most of the decoder backward; one
            # bucket for all layers keeps the first split at the end of the layer loop
            self.eng.merged_layer_bucket = bool(self.pipeline and self.enc_eng is None)
        fp = self.eng.fp
        dec = list(self.eng.grad_buckets())
        bl = [(fp, [r]) for r in dec]
        if self.enc_eng is not None:
            bl.append((fp, _complement(dec, fp.grad.numel())))
            bl += [(self.enc_eng.fp, [r]) for r in self.enc_eng.grad_buckets()]
        self._buckets = bl

    def enable_encoder_finetune(self, startingLayer):
        """train.py:160-166: from this step on, children[startingLayer:] of the encoder train
        with their own Adam (encoder_lr); the captured graph is rebuilt on the next step."""
        self.encoder.fine_tune(fine_tune=True, startingLayer=startingLayer)
        self.flush()
        self.enc_eng = self.encoder.engine() if _trainable(self.encoder) else None
        self._plan_buckets()
        self._graph = None
        self._pipe = None
        self._seq_store = {}
        self._seq_T = None
        rel = getattr(self.encoder, "release_retired", None)
        if rel is not None:  # the graphs that pointed into superseded weight packs are gone
            rel()

    _SEQ_FIELDS = ("_graph", "_inputs", "_metrics", "_feat_slot", "_enc_saved", "_feat_meta", "_seed_ctr")

    def bucket_T(self, caps, caplens, max_caplen=None):
        """Steps the LSTM runs for this batch: the next multiple of 8 >= its longest decode length
        (caplen - 1); positions the Transformer runs: the next multiple of 8 >= its longest caption.
        None (= all of L) when that is not known on the host or length buckets are off."""
        if not self.len_buckets:
            return None
        if max_caplen is None:
            if caplens.device.type != "cpu":
                return None
            max_caplen = int(caplens.max())
        L = caps.size(1)
        if not self.lstm:
            T = max(8, (int(max_caplen) + 7) // 8 * 8)
            return None if T >= L else T
        T = max(8, (int(max_caplen) - 1 + 7) // 8 * 8)
        return None if T >= L - 1 else T

    def _select_seq(self, T):
        """Make bucket T's captured sequential step (graph, static inputs, metrics) current."""
        if T == self._seq_T:
            return
        self._seq_store[self._seq_T] = {f: getattr(self, f, None) for f in self._SEQ_FIELDS}
        for f, v in self._seq_store.get(T, {f: None for f in self._SEQ_FIELDS}).items():
            setattr(self, f, v)
        if self._seed_ctr is not None:  # that bucket's graphs advance their own counter
            K.set_seed_counter(self._seed_ctr)
        self._seq_T = T

    def _encode(self, imgs):
        self.encoder.train()
        with torch.no_grad(), K.workspace_slot(1 if self.pipeline else 0):
            return self.encoder(imgs)

    def _enc_part(self, imgs):
        """Encoder half of the step: (features, saved state of the fine-tuned children or None)."""
        self.encoder.train()
        self.decoder.train()
        if self.enc_eng is not None:
            return self.enc_eng.forward(imgs)
        return self._encode(imgs), None

    def _fwd_bwd(self, imgs, caps, caplens):
        feats, es = self._enc_part(imgs)
        self._feat_meta = (tuple(feats.shape), feats.dtype)
        return self._dec(feats, caps, caplens, es)

    def _dec(self, feats, caps, caplens, es=None, mid=None):
        self.decoder.train()
        if self.lstm:
            s = self.eng.forward(feats, caps, caplens, fixed_T=self._cur_T if self._cur_T else True, alphaC=self.alphaC)
        else:
            if self._cur_T:  # length bucket: the first _cur_T positions (bucket_T)
                caps = caps[:, :self._cur_T]
            s = self.eng.forward(feats, caps, caplens, pad_id=self.pad_id)
        if mid is not None:
            mid()
        hook = self._buckets is not None and self._hook_mode is not None
        kw = {"bucket_hook": self._bucket_hook} if hook else {}
        self._next_bucket = 0
        if es is not None:
            # fine-tuned encoder: the decoder's remaining gradients are final once its backward is
            # done; their all-reduce runs on the comm stream while the encoder children's
            # backward runs, which in turn hands over its ~25 MiB buckets as its blocks finish
            # (trainMultiGPU.py:233-235,256,384: DDP's reducer overlaps the buckets with the rest
            # of the backward)
            self.eng.backward(s, want_denc=True, **kw)
            if hook:
                self._bucket_hook()
            self.enc_eng.backward(es, s["denc"].reshape(feats.shape), **kw)
        else:
            self.eng.backward(s, **kw)
        if hook and self._hook_mode == "eager":
            self._issued = self._next_bucket
        return s["metrics"]

    # ---- bucketed gradient all-reduce --------------------------------------------------------
    def _reduce_ranges(self, fp, ranges):
        """All-reduce (sum) fp.grad[lo:hi] for each range on the communication stream, ordered
        after the current stream's work so far (every collective of the step goes through that
        one stream, in the same order on every rank)."""
        g = fp.grad
        if self._comm is None:
            for lo, hi in ranges:
                if hi > lo:
                    dist.all_reduce(g[lo:hi], op=dist.ReduceOp.SUM, group=self.pg)
            return
        self._comm.wait_stream(torch.cuda.current_stream(g.device))
        with torch.cuda.stream(self._comm):
            for lo, hi in ranges:
                if hi > lo:
                    dist.all_reduce(g[lo:hi], op=dist.ReduceOp.SUM, group=self.pg)

    def _reduce_bucket(self, k):
        fp, ranges = self._buckets[k]
        self._reduce_ranges(fp, ranges)

    def _bucket_hook(self):
        k = self._next_bucket
        self._next_bucket += 1
        if self._hook_mode == "eager":
            self._reduce_bucket(k)
        elif self._hook_mode == "split":
            self._split()

    def _begin_split_capture(self, pool=None, join=None):
        """Capture the step as one graph per bucket hook + 1 (world > 1): the hooks end a graph
        and begin the next in the same pool; returns the list the graphs are appended to.
        ``join``: streams to join at the first split (forked branches of the first graph)."""
        graphs = [torch.cuda.CUDAGraph()]
        joined = []

        def split():
            cur = torch.cuda.current_stream()
            if not joined:
                for st in (join or ()):
                    K.join(cur, st)
                joined.append(True)
            K.assert_joined("split capture")
            graphs[-1].capture_end()
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=graphs[0].pool())
            graphs.append(g)
        self._split = split
        self._hook_mode = "split"
        graphs[0].capture_begin(pool=pool)
        return graphs

    def _end_split_capture(self, graphs):
        self._hook_mode = None
        self._split = None
        K.assert_joined("split capture")
        graphs[-1].capture_end()
        return tuple(graphs)

    def _replay(self, g):
        if isinstance(g, _SeqGraphs):  # encoder half, then decoder half
            g.enc.replay()
            self._replay(g.dec)
            return
        if isinstance(g, tuple):  # split step: bucket i reduced between graphs i and i + 1
            for i, gi in enumerate(g):
                gi.replay()
                if i + 1 < len(g):
                    self._reduce_bucket(i)
            self._issued = len(g) - 1
        else:
            g.replay()

    def _capture(self, imgs, caps, caplens, warmup=2):
        dev = imgs.device
        self._seed_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        K.set_seed_counter(self._seed_ctr)
        self._inputs = (imgs.clone(), caps.clone(), caplens.clone())
        # first-touch allocations and one-time kernel setup, on the capturing stream itself: with
        # the warm-up on a separate stream the captured sequential step faulted on replays after
        # allocator activity (C4 --no-pipeline, C5)
        for _ in range(warmup):
            self._fwd_bwd(*self._inputs)
        torch.cuda.synchronize(dev)
        # the encoder half as its own graph, writing the features into a buffer allocated
        # outside the captures; the decoder half (+ the fine-tuned encoder's backward) reads it.
        # One graph of the whole step, the decoder reading the encoder's output tensor inside
        # the graph's own pool, faulted on replays that followed allocator activity (C4
        # --no-pipeline, C5; tools/probe/capture_bisect.py: the encoder-only, decoder-only and
        # two-graph captures replay cleanly after the regular pool is overwritten)
        shape, dtype = self._feat_meta
        self._feat_slot = torch.empty(shape, dtype=dtype, device=dev)
        ge = torch.cuda.CUDAGraph()
        with torch.cuda.graph(ge):
            self._seed_ctr.add_(1)
            feats, es = self._enc_part(self._inputs[0])
            self._feat_slot.copy_(feats)
            K.assert_joined("encoder graph")
        self._enc_saved = es  # the fine-tuned children's activations live in ge's pool
        if self._buckets is not None:  # decoder half split at the bucket hooks (DDP)
            cap = torch.cuda.Stream(device=dev)
            cap.wait_stream(torch.cuda.current_stream(dev))
            torch.cuda.synchronize(dev)
            with torch.cuda.stream(cap):
                gs = self._begin_split_capture()
                self._metrics = self._dec(self._feat_slot, self._inputs[1], self._inputs[2], es)
                gs = self._end_split_capture(gs)
            torch.cuda.current_stream(dev).wait_stream(cap)
            self._graph = _SeqGraphs(ge, gs)
            return
        gd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gd):
            self._metrics = self._dec(self._feat_slot, self._inputs[1], self._inputs[2], es)
            K.assert_joined("decoder graph")
        self._graph = _SeqGraphs(ge, gd)

    # ---- encoder / decoder pipeline ------------------------------------------------------------
    def _pipe_buffers(self, imgs, caps, caplens):
        """Static inputs of the pipelined schedule, shared by every length bucket's graphs: the
        image batch being encoded, two caption / length slots and (on the first capture) two
        feature slots; one device seed counter."""
        dev = imgs.device
        self._seed_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        K.set_seed_counter(self._seed_ctr)
        self._pipe = dict(side=torch.cuda.Stream(device=dev), i=0, img=imgs.clone(),
                          caps=[caps.clone(), caps.clone()], lens=[caplens.clone(), caplens.clone()],
                          T=[None, None], feats=None, sets={})

    def _pipe_capture(self, T, warmup=2):
        """Graphs of the pipelined step that decode a batch of length bucket T (slot parity k:
        encode the new batch into slot k, train on slot 1 - k)."""
        P = self._pipe
        dev = P["img"].device
        side = P["side"]
        main = torch.cuda.current_stream(dev)
        self._cur_T = T
        side.wait_stream(main)
        with torch.cuda.stream(side):  # first-touch allocations and one-time kernel setup
            for _ in range(warmup):
                f = self._encode(P["img"])
                self._dec(f, P["caps"][0], P["lens"][0])
        main.wait_stream(side)
        if P["feats"] is None:
            P["feats"] = [torch.empty_like(f), torch.empty_like(f)]
        S = dict(graphs=[], metrics=[])
        P["sets"][T] = S
        pool = None
        for k in (0, 1):  # graph k: encode the new batch into slot k, train on slot 1-k
            split = self._buckets is not None
            cap = torch.cuda.Stream(device=dev)
            cap.wait_stream(main)
            torch.cuda.synchronize(dev)
            with torch.cuda.stream(cap):
                if split:  # one graph per bucket + 1; the encoder branch joins the first at its end
                    gs = self._begin_split_capture(pool, join=(side,))
                else:
                    g = torch.cuda.CUDAGraph()
                    g.capture_begin(pool=pool)
                try:
                    self._seed_ctr.add_(1)
                    cur = torch.cuda.current_stream(dev)

                    def fork(k=k, cur=cur):
                        K.fork(side, cur)
                        with torch.cuda.stream(side):
                            P["feats"][k].copy_(self._encode(P["img"]))
                    if PIPE_FORK != "bwd":
                        fork()
                    m = self._dec(P["feats"][1 - k], P["caps"][1 - k], P["lens"][1 - k],
                                  mid=fork if PIPE_FORK == "bwd" else None)
                    K.join(cur, side)
                except BaseException:
                    self._hook_mode, self._split = None, None
                    _abandon_capture(gs[-1] if split else g, (side,))
                    raise
                if split:
                    g = self._end_split_capture(gs)
                else:
                    K.assert_joined("pipelined step graph")
                    g.capture_end()
            main.wait_stream(cap)
            pool = g[0].pool() if split else g.pool()
            S["graphs"].append(g)
            S["metrics"].append(m)

    def _pipe_step(self, imgs, caps, caplens, T=None):
        """Returns the metrics tensor of the previous batch (None on the first call).  T: this
        batch's length bucket (decoded on the next call)."""
        if not self.graph:
            main = torch.cuda.current_stream()
            if self._pipe is None:
                self._pipe = dict(side=torch.cuda.Stream(device=imgs.device), pending=None)
            P = self._pipe
            P["side"].wait_stream(main)
            with torch.cuda.stream(P["side"]):
                feats = self._encode(imgs)
            self._hook_mode = "eager"
            m = None
            if P["pending"] is not None:
                self._cur_T = P["pending"][3]
                m = self._dec(*P["pending"][:3])
            self._hook_mode = None
            main.wait_stream(P["side"])
            feats.record_stream(main)
            P["pending"] = (feats, caps, caplens, T)
            return m
        if self._pipe is None:
            self._pipe_buffers(imgs, caps, caplens)
        P = self._pipe
        k = P["i"] % 2
        if any(d.shape != s_.shape or d.dtype != s_.dtype for d, s_ in ((P["img"], imgs), (P["caps"][k], caps),
                                                                        (P["lens"][k], caplens))):
            # a batch of another shape (the last, partial batch of an epoch): finish the batch in
            # flight, then this one with eager launches, sequentially
            self.flush()
            self._cur_T = T
            return self._eager(imgs, caps, caplens)
        m = None
        if P["i"] > 0 and P["T"][1 - k] not in P["sets"]:
            self._pipe_capture(P["T"][1 - k])  # first batch of this length bucket to be decoded
        for dst, src in ((P["img"], imgs), (P["caps"][k], caps), (P["lens"][k], caplens)):
            dst.copy_(src, non_blocking=True)
        if P["i"] == 0:
            f = self._encode(P["img"])
            if P["feats"] is None:
                P["feats"] = [torch.empty_like(f), torch.empty_like(f)]
            P["feats"][k].copy_(f)
        else:
            S = P["sets"][P["T"][1 - k]]
            self._replay(S["graphs"][k])
            m = S["metrics"][k]
        P["T"][k] = T
        P["i"] += 1
        return m

    def flush(self):
        """Pipeline mode: train on the last batch handed to step() (no-op otherwise)."""
        P = self._pipe
        if not self.pipeline or P is None:
            return None
        self._hook_mode = "eager"
        if not self.graph:
            if P["pending"] is None:
                self._hook_mode = None
                return None
            self._cur_T = P["pending"][3]
            m = self._dec(*P["pending"][:3])
            P["pending"] = None
        else:
            if P["i"] == 0:
                self._hook_mode = None
                return None
            j = (P["i"] - 1) % 2
            self._cur_T = P["T"][j]
            m = self._dec(P["feats"][j], P["caps"][j], P["lens"][j])
            P["i"] = 0
        self._hook_mode = None
        return self._update(m)

    def step(self, imgs, caps, caplens, max_caplen=None):
        """One train step on a batch.  ``max_caplen``: the batch's longest caption length when
        the caller knows it on the host (else read from CPU caplens, else L is assumed)."""
        T = self.bucket_T(caps, caplens, max_caplen)
        if self.pipeline and self.enc_eng is None:
            m = self._pipe_step(imgs, caps, caplens, T)
            return None if m is None else self._update(m)
        self._cur_T = T
        if not self.graph:
            m = self._eager(imgs, caps, caplens)
        else:
            self._select_seq(T)
            if self._graph is None:
                self._capture(imgs, caps, caplens)
            if any(d.shape != s_.shape or d.dtype != s_.dtype for d, s_ in zip(self._inputs, (imgs, caps, caplens))):
                # a batch of another shape (the last, partial batch of an epoch): eager launches
                return self._update(self._eager(imgs, caps, caplens))
            for dst, src in zip(self._inputs, (imgs, caps, caplens)):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src, non_blocking=True)
            self._replay(self._graph)
            m = self._metrics
        return self._update(m)

    def _eager(self, imgs, caps, caplens):
        self._hook_mode = "eager"
        try:
            return self._fwd_bwd(imgs, caps, caplens)
        finally:
            self._hook_mode = None

    def _update(self, m):
        """DDP gradient average, clip + Adam, metric reduction (trainMultiGPU.py:384-403).

        m = [loss, tokens, top-5 hits, 1/tokens, hand-off errors]; m[4] counts the persistent LSTM
        recurrences' timed-out hand-offs.  Such a step's gradients are invalid: the Adam kernels
        read the (rank-summed) error word on the device and leave every parameter and moment as
        it was, the step's loss reads NaN and drain_metrics() raises (decoder.py:100-111 must
        never degrade silently).  One rank: the step's metric vector is logged as is (one copy,
        reduced on the host at drain time); DDP: the reduceLossAndTokens / accuracy sums across
        ranks (trainMultiGPU.py:96-108, 398-403), reduced before the update so every rank skips
        the same steps."""
        fp = self.eng.fp
        if not self.ddp:
            red = m.clone()
        else:
            zero = torch.zeros((), device=m.device, dtype=m.dtype)
            red = torch.stack([m[0] * m[1], m[1], m[2], zero, m[4] if m.numel() > 4 else zero])
            dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.pg)
            red[0] = red[0] / red[1]  # global token-weighted mean loss, back in m's layout
        skip = red[4:5] if red.numel() > 4 else None
        if self.ddp:
            # the buckets issued during the backward are in flight on the comm stream; the ranges
            # none of them covers follow on the same stream, then clip + Adam wait for all of it
            issued = self._buckets[:self._issued] if self._buckets else []
            self._issued = 0
            flats = [fp] + ([self.enc_eng.fp] if self.enc_eng is not None else [])
            for f in flats:
                done = [r for bf, rs in issued if bf is f for r in rs]
                self._reduce_ranges(f, _complement(done, f.grad.numel()))
            if self._comm is not None:
                torch.cuda.current_stream(fp.grad.device).wait_stream(self._comm)
        fp.adam_step(self.decoder_lr, self.grad_clip, grad_div=float(self.world), skip=skip)
        if self.enc_eng is not None:
            efp = self.enc_eng.fp
            efp.adam_step(self.encoder_lr, self.grad_clip, grad_div=float(self.world), skip=skip)
            upd = getattr(self.encoder, "weights_updated", None)
            if upd is not None:  # packed copies of the fine-tuned children go stale
                upd()
        self._metric_log.append(red)
        return red

    # -- checkpoint I/O (checkpoint.py; utils.py:195-224, train.py:118-147) ------------------
    def optimizers(self):
        """(encoderOptimizer, decoderOptimizer) as torch.optim.Adam state dicts in the reference's
        parameter order (None for a frozen encoder) -- the values save_checkpoint stores."""
        from . import checkpoint as ck
        dec = ck.optimizer_state_dict(self.eng.fp, ck.trainable_parameters(self.decoder), self.decoder_lr)
        enc = None
        if self.enc_eng is not None:
            enc = ck.optimizer_state_dict(self.enc_eng.fp, ck.trainable_parameters(self.encoder), self.encoder_lr)
        return enc, dec

    def load_optimizers(self, decoderOptimizer, encoderOptimizer=None):
        """Resume (train.py:135-143): Adam moments, step counts and learning rates from the
        reference-layout state dicts (the model weights are loaded with load_state_dict)."""
        from . import checkpoint as ck
        self.decoder_lr = ck.load_optimizer_state_dict(self.eng.fp, ck.trainable_parameters(self.decoder),
                                                       decoderOptimizer)
        if encoderOptimizer is not None:
            if self.enc_eng is None:
                raise ValueError("encoder optimizer state given but the encoder is frozen")
            self.encoder_lr = ck.load_optimizer_state_dict(self.enc_eng.fp, ck.trainable_parameters(self.encoder),
                                                           encoderOptimizer)

    def drain_metrics(self):
        """(globalLoss, tokens, top5 %) per logged step, like reduceLossAndTokens + accuracy."""
        if not self._metric_log:
            return []
        r = torch.stack([m if m.numel() > 4 else torch.cat([m, m.new_zeros(5 - m.numel())])
                         for m in self._metric_log]).double().cpu()
        self._metric_log = []
        failed = int((r[:, 4] > 0).sum())
        if failed:
            raise RuntimeError(f"persistent LSTM recurrence: a workgroup hand-off timed out in {failed} of the "
                               f"{r.shape[0]} logged steps (error word set); their updates are invalid")
        return [(float(a), float(b), float(c / b * 100.0)) for a, b, c in r[:, :3]]
