"""Entry points keep the reference's CLI (train.py:59-65) and produce COCO-shaped batches."""
import train


def test_cli_flags_match_reference():
    a = train.parse(["--teacherForcing", "--lstmDecoder", "--startingLayer", "7", "--encoderLr", "3e-4"])
    assert a.teacherForcing and a.lstmDecoder and a.startingLayer == 7 and abs(a.encoderLr - 3e-4) < 1e-12
    assert a.checkpoint is None and a.embeddingName is None
    d = train.parse([])
    assert d.startingLayer == 5 and d.encoderLr == 1e-4 and not d.teacherForcing


def test_synthetic_batches_shape():
    imgs, caps, lens = next(train.synthetic_loader(1, 2, "cpu"))
    assert imgs.shape == (2, 3, 224, 224) and caps.shape == (2, 52) and lens.shape == (2, 1)
    assert (caps[:, 0] == train.VOCAB - 2).all() and (caps[:, -1] == train.VOCAB - 1).all()
    assert int(lens[0]) == 52


def test_testpy_cli_and_results_name_match_reference():
    """test.py:63-68 flags and the results CSV names of test.py:128-131."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("imgcap_testpy", os.path.join(root, "test.py"))
    testpy = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(testpy)
    a = testpy.parse(["--checkpoint", "x.pth.tar", "--lstmDecoder", "--startingLayer", "7"])
    assert a.checkpoint == "x.pth.tar" and a.lstmDecoder and a.startingLayer == 7 and a.embeddingName is None
    assert testpy.results_name(True, 7, None) == "test-lstmDecoder-TeacherForcing-Finetuning7.csv"
    assert testpy.results_name(False, None, None) == "test-TransformerDecoder-TeacherForcing-FinetuningNone-None.csv"


def test_trainMultiGPU_cli_accepts_reference_launch_line():
    """README.md:33 launches ``srun python3 trainMultiGPU.py --port 29500 --teacherForcing``;
    trainMultiGPU.py:63-70: --port, startingLayer default 7."""
    import shlex
    import trainMultiGPU
    argv = shlex.split("srun python3 trainMultiGPU.py --port 29500 --teacherForcing")[3:]
    a = trainMultiGPU.parse(argv)
    assert a.port == "29500" and a.teacherForcing and a.startingLayer == 7 and not a.lstmDecoder
    assert a.encoderLr == 1e-4 and a.checkpoint is None and a.embeddingName is None
    assert trainMultiGPU.parse(["--port", "29611"]).port == "29611"
    assert trainMultiGPU.EARLY_STOP == 40


def test_trainMultiGPU_rendezvous_env():
    """SLURM: MASTER_PORT := --port (trainMultiGPU.py:148); torchrun: its own port stays."""
    import trainMultiGPU
    env = {"SLURM_PROCID": "3", "SLURM_NTASKS": "8", "SLURM_LOCALID": "3", "MASTER_PORT": "1"}
    assert trainMultiGPU.dist_env("29611", env) == (3, 8, 3)
    assert env["MASTER_PORT"] == "29611" and env["MASTER_ADDR"] == "127.0.0.1"
    env = {"RANK": "1", "WORLD_SIZE": "2", "LOCAL_RANK": "1", "MASTER_PORT": "40000", "MASTER_ADDR": "10.0.0.1"}
    assert trainMultiGPU.dist_env("29500", env) == (1, 2, 1)
    assert env["MASTER_PORT"] == "40000" and env["MASTER_ADDR"] == "10.0.0.1"


class _FakeTrainer:
    """The attributes run_epochs touches; records the lr each epoch trains with."""

    def __init__(self):
        self.decoder_lr, self.encoder_lr, self.enc_eng, self.log = 1e-4, 1e-4, None, []

    def enable_encoder_finetune(self, startingLayer):
        self.enc_eng = object()

    def step(self, *a, **k):
        pass

    def flush(self):
        pass

    def drain_metrics(self):
        self.log.append((self.decoder_lr, self.encoder_lr, self.enc_eng is not None))
        return [(1.0, 1.0, 1.0)]


class _Val:
    dataset = type("D", (), {"wordMap": {}})()


def _epochs_worker(rank, world, initfile, outdir, early_stop, epochs, fine_tune_from):
    import json
    import os
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + initfile, rank=rank, world_size=world)
    args = train.parse(["--teacherForcing", "--steps", "0", "--epochs", str(epochs),
                        "--fineTuneFromEpoch", str(fine_tune_from), "--encoderLr", "3e-4"])
    tr = _FakeTrainer()
    nval = [0]

    def validate_fn(*a, **k):  # BLEU-4 improves once, then never again
        nval[0] += 1
        return 0, 0, 0, 0, 0, (0.5 if nval[0] == 1 else 0.1)

    enc = dec = torch.nn.Linear(1, 1)
    esi, _ = train.run_epochs(args, enc, dec, tr, None, torch.device("cpu"), rank=rank, world=world,
                              log=lambda *a, **k: None, early_stop=early_stop,
                              val=lambda a: _Val(), validate_fn=validate_fn)
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump({"esi": esi, "epochs": tr.log, "validated": nval[0]}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_run_epochs_two_ranks_agree_on_decay_and_stop(tmp_path):
    """only rank 0 validates; epochsSinceImprovement is broadcast so both ranks decay
    the lr at the same epochs and stop together (trainMultiGPU.py:259-264, 332-334).  The
    encoder lr is not decayed before the encoder optimizer exists and starts at --encoderLr."""
    import json
    import os
    import torch.multiprocessing as mp
    epochs, stop, ft = 30, 17, 5
    mp.spawn(_epochs_worker, args=(2, os.path.join(str(tmp_path), "init"), str(tmp_path), stop, epochs, ft),
             nprocs=2, join=True)
    r = [json.load(open(os.path.join(str(tmp_path), f"r{k}.json"))) for k in range(2)]
    assert r[0]["epochs"] == r[1]["epochs"] and r[0]["esi"] == r[1]["esi"] == stop
    assert r[0]["validated"] == len(r[0]["epochs"]) and r[1]["validated"] == 0
    # epoch 0 improves; epochs 1.. do not: esi after epoch e = e, so training stops before epoch 18
    assert len(r[0]["epochs"]) == stop + 1
    dec_lr = [e[0] for e in r[0]["epochs"]]
    enc_lr = [e[1] for e in r[0]["epochs"]]
    # decays at the start of epochs with esi in {8, 16} -> epochs 9 and 17
    assert all(abs(dec_lr[e] - 1e-4 * 0.8 ** ((e >= 9) + (e >= 17))) < 1e-15 for e in range(stop + 1))
    assert all(abs(enc_lr[e] - 3e-4 * 0.8 ** ((e >= 9) + (e >= 17))) < 1e-15 for e in range(ft, stop + 1))
    assert [e[2] for e in r[0]["epochs"]] == [e >= ft for e in range(stop + 1)]
