"""Multi-GPU (one process per GPU) teacher-forced training entry point, trainMultiGPU.py's
counterpart: SLURM variables (trainMultiGPU.py:144-146) or torchrun's RANK / WORLD_SIZE /
LOCAL_RANK, backend "nccl" (= RCCL over xGMI), DDP-equivalent gradient averaging inside
``TeacherForcedTrainer`` (bucketed all-reduces of the flat gradient buffer as the backward produces
the buckets, like DDP's reducer) and the
``reduceLossAndTokens`` metric reduction (:96-108).

    srun python3 trainMultiGPU.py --port 29500 --teacherForcing        (the reference's launch line)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 trainMultiGPU.py \
        --teacherForcing --encoder base --batchSize 32

CLI: trainMultiGPU.py:63-70 (``--port``, ``--startingLayer`` default 7) plus this build's
additions shared with train.py; early stop after 40 epochs without improvement (:259).
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import train  # noqa: E402  (model construction, CLI and the epoch loop are shared)


EARLY_STOP = 40  # trainMultiGPU.py:259 (train.py uses 20)


def parse(argv=None):
    return train.make_parser(multi_gpu=True).parse_args(argv)


def dist_env(port, environ=None):
    """(rank, world, local) from SLURM (trainMultiGPU.py:144-146) or torchrun's variables, and
    the rendezvous address: under SLURM MASTER_PORT comes from --port (:148); under torchrun its
    own MASTER_PORT stays (the workers join torchrun's store there)."""
    env = os.environ if environ is None else environ
    if "SLURM_PROCID" in env and "RANK" not in env:
        rank, world, local = (int(env[k]) for k in ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"))
        env["MASTER_PORT"] = str(port)
    else:
        rank, world, local = (int(env.get(k, d)) for k, d in (("RANK", 0), ("WORLD_SIZE", 1), ("LOCAL_RANK", 0)))
        env.setdefault("MASTER_PORT", str(port))
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return rank, world, local


def setup_distributed(port="29500"):
    """trainMultiGPU.py:144-160 (SLURM) or torchrun environment."""
    rank, world, local = dist_env(port)
    torch.cuda.set_device(local)
    device = torch.device(f"cuda:{local}")
    dist.init_process_group("nccl", init_method="env://", world_size=world, rank=rank, device_id=device)
    return rank, local, world, device


def main(argv=None):
    args = parse(argv)
    if not args.teacherForcing:
        raise NotImplementedError("non-teacher-forced training is outside the accelerated path (SURVEY.md §8f)")
    rank, local, world, device = setup_distributed(args.port)
    torch.manual_seed(42 + rank)
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    encoder, decoder, ck = train.build_models(args, device)
    trainer = TeacherForcedTrainer(encoder, decoder, lstm=args.lstmDecoder, decoder_lr=train.decoderLr,
                                   encoder_lr=args.encoderLr, grad_clip=train.gradClip, alphaC=train.alphaC,
                                   graph=True, pipeline=not args.noPipeline)
    log = print if rank == 0 else (lambda *a, **k: None)
    # trainMultiGPU.py: encoder fine-tuned (and DDP-averaged) from epoch 20; rank 0 checkpoints
    train.run_epochs(args, encoder, decoder, trainer, ck, device, rank=rank, log=log, world=world,
                     early_stop=EARLY_STOP)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
