"""Fused train step (train.py:251-299): eager launches vs HIP-graph replay, and the device
seed counter that keeps dropout / stochastic-depth masks fresh across replays."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(dev, decoder, dropout, sd_off, dtype=torch.float32, starting_layer=None):
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    torch.manual_seed(5)
    enc = Encoder(variant="tiny", compute_dtype=dtype)
    if starting_layer is None:
        enc.fine_tune(False)
    else:
        enc.fine_tune(True, startingLayer=starting_layer)
    if sd_off:
        for m in enc.modules():
            if hasattr(m, "sd_prob"):
                m.sd_prob = 0.0
    if decoder == "lstm":
        dec = DecoderWithAttention(attention_dim=64, embed_dim=64, decoder_dim=64, vocab_size=120, device=dev,
                                   encoder_dim=768, dropout=dropout, compute_dtype=dtype)
    else:
        dec = TransformerDecoder(embed_dim=128, decoder_dim=128, vocab_size=120, maxLen=20, device=dev,
                                 wordMap=None, pretrained_embeddings_path=None, fine_tune_embeddings=True,
                                 dropout=dropout, encoder_dim=768, num_heads=2, num_layers=2,
                                 compute_dtype=dtype)
    return enc.to(dev), dec.to(dev)


def _batch(dev, i, B=4, L=20, V=120, hw=64):
    g = torch.Generator().manual_seed(100 + i)
    img = torch.randn(B, 3, hw, hw, generator=g)
    caps = torch.randint(1, V - 2, (B, L), generator=g)
    caps[:, 0] = V - 2
    lens = torch.tensor([L, 15, 11, 7])[:B]
    for b in range(B):
        caps[b, lens[b] - 1] = V - 1
        caps[b, lens[b]:] = 0
    return img.to(dev), caps.to(dev), lens.view(B, 1).to(dev)


@pytest.mark.parametrize("decoder", ["lstm", "transformer"])
def test_graph_replay_matches_eager(hip_device, decoder):
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    runs = []
    for graph in (False, True):
        enc, dec = _models(hip_device, decoder, dropout=0.0, sd_off=True)
        tr = TeacherForcedTrainer(enc, dec, lstm=decoder == "lstm", graph=graph)
        for i in range(3):
            tr.step(*_batch(hip_device, i))
        runs.append((tr.drain_metrics(), tr.eng.fp.flat.clone()))
        K.set_seed_counter(None)
    (m_e, p_e), (m_g, p_g) = runs
    for a, b in zip(m_e, m_g):
        assert abs(a[0] - b[0]) < 1e-5 * abs(a[0]) and a[1] == b[1] and abs(a[2] - b[2]) < 1e-3
    # no float atomics anywhere in the step (the embedding gradient sums its rows in position
    # order): graph replay and eager launches run the same kernels in the same order
    assert torch.equal(p_g, p_e)


@pytest.mark.parametrize("decoder", ["lstm", "transformer"])
def test_train_step_bitwise_repeatable(hip_device, decoder):
    """Deterministic mode (the reference's test.py:12-24 seeds everything and its
    results/checkingReproducibility shows ~1e-7 run-to-run drift): two trainers from the same
    state over the same batches end with bitwise-identical parameters, Adam moments and metrics,
    dropout and drop path active."""
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    runs = []
    for _ in range(2):
        enc, dec = _models(hip_device, decoder, dropout=0.5, sd_off=False)
        tr = TeacherForcedTrainer(enc, dec, lstm=decoder == "lstm", graph=True)
        for i in range(3):
            tr.step(*_batch(hip_device, i))
        fp = tr.eng.fp
        runs.append((tr.drain_metrics(), fp.flat.clone(), fp.m.clone(), fp.v.clone()))
        K.set_seed_counter(None)
    (m1, *a), (m2, *b) = runs
    assert m1 == m2
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_graph_replays_draw_fresh_masks(hip_device):
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    enc, dec = _models(hip_device, "lstm", dropout=0.5, sd_off=False)
    tr = TeacherForcedTrainer(enc, dec, lstm=True, graph=True, decoder_lr=0.0)
    x = _batch(hip_device, 0)
    for _ in range(3):
        tr.step(*x)
    losses = [m[0] for m in tr.drain_metrics()]
    # lr 0: the only thing that changes between replays is the dropout / drop-path masks
    assert len(set(losses)) == 3, losses
    # the same counter value reproduces the same masks
    tr._seed_ctr.fill_(0)
    tr.step(*x)
    again = tr.drain_metrics()[0][0]
    assert again == losses[0]
    K.set_seed_counter(None)


@pytest.mark.parametrize("graph,bucketed", [(False, True), (True, True), (True, False)])
def test_trainer_ddp2_hip_matches_reference_trainMultiGPU(hip_device, tmp_path, graph, bucketed):
    """Two ranks (gloo, sharing the one GPU) through the HIP engine vs the reference's 2-rank
    trainMultiGPU step (tests/golden/ddp2_lstm): eager (early bucket reduced from the backward's
    hook on the comm stream) and graph replay (the step split into two graphs around it)."""
    import ddp_util
    ddp_util.check(ddp_util.run("hip", tmp_path, graph=graph, bucketed=bucketed))


@pytest.mark.parametrize("decoder", ["lstm", "transformer"])
@pytest.mark.parametrize("graph", [False, True])
def test_pipelined_trainer_matches_sequential(hip_device, decoder, graph):
    """pipeline=True runs the frozen encoder of batch i on a second stream beside the decoder
    step of batch i-1: the metrics (one step late) and the parameter updates must be exactly
    those of the sequential trainer."""
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    runs = []
    for pipe in (False, True):
        enc, dec = _models(hip_device, decoder, dropout=0.0, sd_off=True)
        tr = TeacherForcedTrainer(enc, dec, lstm=decoder == "lstm", graph=graph, pipeline=pipe)
        outs = [tr.step(*_batch(hip_device, i)) for i in range(4)]
        if pipe:
            assert outs[0] is None
            tr.flush()
        runs.append((tr.drain_metrics(), tr.eng.fp.flat.clone()))
        K.set_seed_counter(None)
    (m_s, p_s), (m_p, p_p) = runs
    assert len(m_s) == len(m_p) == 4
    for a, b in zip(m_s, m_p):
        assert abs(a[0] - b[0]) < 1e-5 * abs(a[0]) and a[1] == b[1] and abs(a[2] - b[2]) < 1e-3
    torch.testing.assert_close(p_p, p_s, rtol=1e-5, atol=5e-6)


@pytest.mark.parametrize("pipeline", [False, True])
def test_bucketed_allreduce_matches_single_collective_over_steps(hip_device, tmp_path, pipeline):
    """Several DDP steps (gloo, 2 ranks on the one GPU) with graph replay, split into two graphs
    around the early bucket (and, pipelined, with the encoder branch joined at the split):
    bitwise the parameters and metrics of one all-reduce after the backward."""
    import ddp_util
    a = ddp_util.run_steps(tmp_path / "a", pipeline, True, True)
    b = ddp_util.run_steps(tmp_path / "b", pipeline, True, False)
    for ra, rb in zip(a, b):
        assert torch.equal(ra["flat"], rb["flat"]) and torch.equal(ra["metrics"], rb["metrics"])
    assert torch.equal(a[0]["flat"], a[1]["flat"])


def _churn(dev, i):
    """Regular-pool allocator activity between replays: blocks of many sizes allocated, filled
    with 0xFF, freed; a few kept (so the next step sees a different layout)."""
    ts = [torch.empty((mb << 20) + 4096 * i, dtype=torch.uint8, device=dev).fill_(255) for mb in (1, 2, 5, 13, 34)]
    ts += [torch.full((n,), -1, dtype=torch.int64, device=dev) for n in (1, 7, 100, 5000) * 4]
    torch.cuda.synchronize(dev)
    return ts[i % 3::3]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_captured_finetune_step_survives_allocator_churn(hip_device, dtype):
    """The captured sequential schedule (encoder graph + decoder graph, the fine-tuned children's
    backward inside the second; what train.py / trainMultiGPU.py run with a fine-tuned encoder,
    and C5) replayed over several steps with deliberate allocator activity between the replays
    (and the eager Adam / metric update): bitwise the parameters, Adam moments and metrics of the
    same steps launched eagerly.  Tiny, fine_tune(True, 7), Transformer decoder, 224x224."""
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    runs = []
    for graph in (False, True):
        enc, dec = _models(hip_device, "transformer", dropout=0.0, sd_off=True, dtype=dtype, starting_layer=7)
        tr = TeacherForcedTrainer(enc, dec, lstm=False, graph=graph)
        assert tr.enc_eng is not None
        keep = []
        for i in range(5):
            keep = _churn(hip_device, i)
            tr.step(*_batch(hip_device, i % 2, B=2, hw=224))
        torch.cuda.synchronize()
        del keep
        e, d = tr.enc_eng.fp, tr.eng.fp
        runs.append((tr.drain_metrics(), d.flat.clone(), d.m.clone(), e.flat.clone(), e.m.clone(), e.v.clone()))
        K.set_seed_counter(None)
    (m_e, *a), (m_g, *b) = runs
    assert m_e == m_g
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("direction", ["FWD", "BWD"])
def test_persistent_lstm_handoff_timeout_raises(hip_device, monkeypatch, direction):
    """A hand-off of the persistent LSTM recurrence that never completes (test knob: U block 0
    skips one publish, csrc/lstm_persist.hip) must not train silently on half-written outputs
    (decoder.py:100-111): the step's error count is set and drain_metrics() raises."""
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    enc, dec = _models(hip_device, "lstm", dropout=0.0, sd_off=True)
    tr = TeacherForcedTrainer(enc, dec, lstm=True, graph=False)
    tr.step(*_batch(hip_device, 0))  # healthy step first
    assert tr.eng._sync is not None  # the persistent recurrences ran
    assert len(tr.drain_metrics()) == 1
    fp = tr.eng.fp
    before = (fp.flat.clone(), fp.m.clone(), fp.v.clone(), fp.shadow)
    monkeypatch.setenv(f"IMGCAP_LSTM_FAULT_{direction}", "2")
    tr.step(*_batch(hip_device, 1))
    monkeypatch.delenv(f"IMGCAP_LSTM_FAULT_{direction}")
    red = tr._metric_log[-1].cpu()  # [loss, tokens, top-5 hits, 1/tokens, hand-off errors]
    assert red[4] > 0
    # the Adam kernel read the error word on the device: the failed step's (invalid) gradients
    # reached neither the parameters nor the moments
    for x, y in zip(before[:3], (fp.flat, fp.m, fp.v)):
        assert torch.equal(x, y)
    with pytest.raises(RuntimeError, match="hand-off timed out"):
        tr.drain_metrics()
    tr.step(*_batch(hip_device, 1))  # the knob is read per launch: clean again
    assert len(tr.drain_metrics()) == 1


@pytest.mark.parametrize("graph", [False, True])
def test_ddp2_transformer_finetuned_encoder_hip(hip_device, tmp_path, graph):
    """Transformer decoder + ConvNeXt-Tiny children[7:] trainable, 2 gloo ranks on the one GPU
    (trainMultiGPU.py:233-235, 256, 384-394): one bucket per decoder layer as its backward ends,
    the decoder's rest beside the encoder backward, the encoder's 25 MiB bucket when its blocks
    are done, the remainder after (eager: from the hooks on the comm stream; graph: between the
    graphs the hooks split the step into); bitwise equal to one collective after the backward,
    and to a single process summing the two shards' gradients."""
    import ddp_ft_util
    a = ddp_ft_util.run_hip(tmp_path / "a", graph, True)
    b = ddp_ft_util.run_hip(tmp_path / "b", graph, False)
    for ra, rb in zip(a, b):
        for k in ra:
            assert torch.equal(ra[k], rb[k]), k
    for k in a[0]:
        assert torch.equal(a[0][k], a[1][k]), k
    dec, enc = ddp_ft_util.expected_hip(hip_device)
    assert torch.equal(a[0]["dec"], dec) and torch.equal(a[0]["enc"], enc)


def test_ddp2_transformer_pipelined_layer_buckets_hip(hip_device, tmp_path):
    """Frozen encoder + Transformer decoder, pipelined captured schedule (C3 / C4 under DDP), 2
    gloo ranks on the one GPU: the per-layer buckets split each step into layers + 1 graphs (the
    encoder branch joined at the first split); bitwise the parameters, Adam moments and metrics
    of one collective after the backward, and the ranks agree."""
    import ddp_ft_util
    a = ddp_ft_util.run_hip(tmp_path / "a", True, True, steps=3, frozen=True)
    b = ddp_ft_util.run_hip(tmp_path / "b", True, False, steps=3, frozen=True)
    for ra, rb in zip(a, b):
        for k in ra:
            assert torch.equal(ra[k], rb[k]), k
    for k in a[0]:
        assert torch.equal(a[0][k], a[1][k]), k


@pytest.mark.parametrize("decoder,pipeline,split", [("lstm", False, False), ("lstm", True, True),
                                                    ("transformer", False, True), ("transformer", True, False)])
def test_captured_step_graphs_hold_only_kernel_nodes(hip_device, monkeypatch, decoder, pipeline, split):
    """Every library launch of the captured step is a KERNEL node: with a memset node in the
    decoder's first half, the split (DDP) schedule faulted on that half's second replay while the
    runtime's graph packet capture was on, and ran clean with it off or with the memsets turned
    into a zeroing kernel (gpurun_out/r3split).  The only non-kernel node allowed
    is torch's own device-to-device copy of the encoder features into the slot the decoder reads."""
    import graph_nodes
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    kept = []
    base = torch.cuda.CUDAGraph

    class Kept(base):
        def __new__(cls, keep_graph=False):
            g = base.__new__(cls, True)
            kept.append(g)
            return g

        def __init__(self, keep_graph=False):
            super().__init__(True)
    monkeypatch.setattr(torch.cuda, "CUDAGraph", Kept)
    enc, dec = _models(hip_device, decoder, 0.1, False)
    tr = TeacherForcedTrainer(enc, dec, lstm=decoder == "lstm", graph=True, pipeline=pipeline)
    if split:  # the DDP split at every bucket hook, reduced over no group (one rank)
        tr._buckets = [(tr.eng.fp, [r]) for r in tr.eng.grad_buckets()]
        tr._reduce_bucket = lambda k: None
    for i in range(3):
        tr.step(*_batch(hip_device, i))
    torch.cuda.synchronize()
    assert kept
    for g in kept:
        nodes = graph_nodes.describe(g.raw_cuda_graph())
        kind = [n.split("] ", 1)[1].split()[0] for n in nodes]
        assert set(kind) <= {"kernel", "memcpy"}, [n for n, k in zip(nodes, kind) if k not in ("kernel", "memcpy")]
        assert kind.count("memcpy") <= 1, [n for n, k in zip(nodes, kind) if k == "memcpy"]


def _len_batch(dev, i, lens, L=40, V=120, hw=64):
    g = torch.Generator().manual_seed(300 + i)
    B = len(lens)
    img = torch.randn(B, 3, hw, hw, generator=g)
    caps = torch.randint(1, V - 2, (B, L), generator=g)
    caps[:, 0] = V - 2
    for b, n in enumerate(lens):
        caps[b, n - 1] = V - 1
        caps[b, n:] = 0
    return img.to(dev), caps.to(dev), torch.tensor(lens).view(B, 1).to(dev), max(lens)


@pytest.mark.parametrize("pipeline", [False, True])
def test_lstm_length_buckets_match_full_steps(hip_device, pipeline):
    """decoder.py:91,100-111: the trainer's length buckets (T = next multiple of 8 >= the longest
    decode length, host-known max caplen) train exactly what L - 1 steps train: the rows past a
    caption's length are masked either way.  Buckets 24, 8, 32, 24 (the last replays the first's
    graph), graphs + pipeline vs the same trainer without buckets."""
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    seqs = [[20, 15, 11, 7], [9, 8, 7, 6], [33, 20, 10, 5], [18, 18, 3, 3], [21, 2, 2, 2]]
    out = []
    for buckets in (False, True):
        enc, dec = _models(hip_device, "lstm", 0.0, True)
        tr = TeacherForcedTrainer(enc, dec, lstm=True, graph=True, pipeline=pipeline, len_buckets=buckets)
        for i, lens in enumerate(seqs):
            img, caps, caplens, mx = _len_batch(hip_device, i, lens)
            assert tr.bucket_T(caps, caplens, mx) == ((mx - 1 + 7) // 8 * 8 if buckets else None)
            tr.step(img, caps, caplens, max_caplen=mx)
        tr.flush()
        torch.cuda.synchronize()
        out.append((tr.eng.fp.flat.detach().cpu().clone(), tr.drain_metrics()))
    (p0, m0), (p1, m1) = out
    assert len(m0) == len(m1) == len(seqs)
    for a, b in zip(m0, m1):
        assert abs(a[0] - b[0]) <= 1e-5 * abs(a[0]) and a[1] == b[1] and abs(a[2] - b[2]) < 1e-6
    assert ((p0 - p1).norm() / p0.norm()).item() < 2e-5  # Adam sign flips at round-off-level grads


@pytest.mark.parametrize("pipeline", [False, True])
def test_transformer_length_buckets_match_full_steps(hip_device, pipeline):
    """transformerDecoder.py:88-108: positions past every caption of the batch are key-padding
    masked and carry no loss rows, so the trainer's Transformer buckets (the first L' = next
    multiple of 8 >= the longest caption positions) train what all L positions train.  Buckets 8,
    16, full, 8 (replaying the first's graphs), 16, with graphs (+ pipeline) vs no buckets."""
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    seqs = [[7, 5, 3, 8], [12, 9, 16, 2], [20, 4, 11, 6], [6, 6, 6, 6], [10, 15, 3, 9]]
    out = []
    for buckets in (False, True):
        enc, dec = _models(hip_device, "transformer", 0.0, True)
        tr = TeacherForcedTrainer(enc, dec, lstm=False, graph=True, pipeline=pipeline, len_buckets=buckets)
        for i, lens in enumerate(seqs):
            img, caps, caplens, mx = _len_batch(hip_device, i, lens, L=20)
            want = (mx + 7) // 8 * 8 if buckets else None
            assert tr.bucket_T(caps, caplens, mx) == (want if want is not None and want < 20 else None)
            tr.step(img, caps, caplens, max_caplen=mx)
        tr.flush()
        torch.cuda.synchronize()
        out.append((tr.eng.fp.flat.detach().cpu().clone(), tr.drain_metrics()))
    (p0, m0), (p1, m1) = out
    assert len(m0) == len(m1) == len(seqs)
    for a, b in zip(m0, m1):
        assert abs(a[0] - b[0]) <= 1e-5 * abs(a[0]) and a[1] == b[1] and abs(a[2] - b[2]) < 1e-6
    assert ((p0 - p1).norm() / p0.norm()).item() < 2e-5  # Adam sign flips at round-off-level grads


def test_eval_after_finetune_step_sees_updated_encoder(hip_device):
    """After a fine-tuned step (EncoderEngine's Adam writes the trainable children through raw
    pointers), the no_grad encoder forward used by validation runs the UPDATED weights: it equals
    a fresh encoder loaded with the updated state_dict (fp32)."""
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    enc, dec = _models(hip_device, "transformer", dropout=0.0, sd_off=True, starting_layer=5)
    imgs = _batch(hip_device, 3, B=2, hw=224)[0]
    enc.eval()
    with torch.no_grad():
        f0 = enc(imgs).clone()  # packs the weights before fine-tuning
    tr = TeacherForcedTrainer(enc, dec, lstm=False, graph=False, encoder_lr=1e-2)
    for i in range(2):
        tr.step(*_batch(hip_device, i, B=2, hw=224))
    torch.cuda.synchronize()
    tr.drain_metrics()
    enc.eval()
    with torch.no_grad():
        f1 = enc(imgs)
    ref = Encoder(variant="tiny", compute_dtype=torch.float32)
    ref.load_state_dict({k: v.detach().clone() for k, v in enc.state_dict().items()})
    ref = ref.to(hip_device).eval()
    ref.fine_tune(False)
    for m in ref.modules():
        if hasattr(m, "sd_prob"):
            m.sd_prob = 0.0
    with torch.no_grad():
        f2 = ref(imgs)
    assert (f1 - f0).abs().max() > 1e-4  # the update is visible
    torch.testing.assert_close(f1, f2, rtol=1e-5, atol=1e-5)
    K.set_seed_counter(None)
