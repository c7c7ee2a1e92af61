"""Checkpoints in the reference's schema, so reference-trained checkpoints resume on the HIP
path and checkpoints written here load in the reference.

  * ``save_checkpoint`` = utils.py:195-224: the same dict keys ('epoch',
    'epochsSinceImprovement', 'bleu-4', 'encoder', 'decoder', 'encoderOptimizer',
    'decoderOptimizer', 'results') and the same file names (``checkpoint_LSTM_Finetuning…`` /
    ``checkpoint_Transformer_Finetuning…`` + a ``BEST_`` copy).
  * Optimizer entries are ``torch.optim.Adam.state_dict()`` dicts: parameter i is the i-th
    entry of ``filter(lambda p: p.requires_grad, module.parameters())`` (train.py:110,114), its
    state {'step', 'exp_avg', 'exp_avg_sq'}.  The build's fused Adam keeps those moments in the
    flat fp32 buffers of ``FlatParams`` (``m``, ``v``); the functions here translate between
    the two layouts by parameter identity.
  * Loading uses ``torch.load(..., weights_only=True)`` (train.py:128 uses weights_only=False;
    the schema holds only tensors and plain Python values, so nothing needs unpickling).
"""
import math
import os
import shutil

import torch

_ADAM_GROUP = dict(weight_decay=0, amsgrad=False, maximize=False, foreach=None, capturable=False,
                   differentiable=False, fused=None, decoupled_weight_decay=False)


def trainable_parameters(module):
    """The parameter list the reference hands to Adam (train.py:110,114)."""
    return [p for p in module.parameters() if p.requires_grad]


def _slices(fp, params):
    name_of = {id(p): n for n, p in fp.params.items()}
    out = []
    for i, p in enumerate(params):
        n = name_of.get(id(p))
        if n is None:
            raise ValueError(f"parameter {i} (shape {tuple(p.shape)}) is not held by this optimizer's flat buffer")
        o, shp = fp.offsets[n]
        out.append((o, math.prod(shp), shp))
    return out


def optimizer_state_dict(fp, params, lr, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam.state_dict() of the fused optimizer over ``fp`` for ``params``."""
    state = {}
    if fp.step_count > 0:
        for i, (o, n, shp) in enumerate(_slices(fp, params)):
            state[i] = {"step": torch.tensor(float(fp.step_count)),
                        "exp_avg": fp.m[o:o + n].view(shp).clone(),
                        "exp_avg_sq": fp.v[o:o + n].view(shp).clone()}
    group = dict(lr=lr, betas=tuple(betas), eps=eps, **_ADAM_GROUP)
    group["params"] = list(range(len(params)))
    return {"state": state, "param_groups": [group]}


def load_optimizer_state_dict(fp, params, sd):
    """Adam state_dict (reference layout) -> the flat moments of ``fp``; returns the group's lr.

    Raises if the parameter count or any moment shape differs (as torch's load_state_dict
    does).  The fused kernel keeps one step count per buffer: parameters stepped a different
    number of times (never the case in train.py, where every trainable parameter gets a
    gradient each step) are rejected."""
    groups = sd["param_groups"]
    ids = [i for g in groups for i in g["params"]]
    if len(ids) != len(params):
        raise ValueError(f"optimizer state has {len(ids)} parameters, the module {len(params)}")
    sl = _slices(fp, params)
    steps = set()
    with torch.no_grad():
        fp.m.zero_()
        fp.v.zero_()
        for k, (o, n, shp) in zip(ids, sl):
            st = sd["state"].get(k)
            if st is None:
                steps.add(0)
                continue
            for key, buf in (("exp_avg", fp.m), ("exp_avg_sq", fp.v)):
                t = st[key]
                if tuple(t.shape) != tuple(shp):
                    raise ValueError(f"{key} of parameter {k}: shape {tuple(t.shape)} != {tuple(shp)}")
                buf[o:o + n].copy_(t.reshape(-1).to(buf))
            steps.add(int(float(st["step"])))
    if len(steps) > 1:
        raise ValueError(f"parameters were stepped different numbers of times {sorted(steps)}; the fused "
                         "optimizer keeps one step count")
    fp.step_count = steps.pop() if steps else 0
    return groups[0]["lr"]


def checkpoint_filename(dataName, lstmDecoder, startingLayer, encoderLr, pretrainedEmbeddingsName):
    """utils.py:216-219."""
    if lstmDecoder is True:
        return 'checkpoint_LSTM_Finetuning' + str(startingLayer) + '_' + str(encoderLr) + '_' + dataName + '.pth.tar'
    return ('checkpoint_Transformer_Finetuning' + str(startingLayer) + '_' + str(encoderLr) + '_' +
            str(pretrainedEmbeddingsName) + '_' + dataName + '.pth.tar')


def _sd(opt):
    if opt is None or isinstance(opt, dict):
        return opt
    return opt.state_dict()


def save_checkpoint(dataName, epoch, epochsSinceImprovement, encoderSaved, decoderSaved, encoderOptimizer,
                    decoderOptimizer, bleu4, isBest, results, lstmDecoder, startingLayer, encoderLr,
                    pretrainedEmbeddingsName, directory="."):
    """utils.py:195-224 (same arguments; optimizers may be state dicts or have ``state_dict()``,
    e.g. ``TeacherForcedTrainer.optimizers()``).  Returns the path written."""
    state = {'epoch': epoch,
             'epochsSinceImprovement': epochsSinceImprovement,
             'bleu-4': bleu4,
             'encoder': encoderSaved,
             'decoder': decoderSaved,
             'encoderOptimizer': _sd(encoderOptimizer),
             'decoderOptimizer': _sd(decoderOptimizer),
             'results': results}
    path = os.path.join(directory, checkpoint_filename(dataName, lstmDecoder, startingLayer, encoderLr,
                                                       pretrainedEmbeddingsName))
    torch.save(state, path)
    if isBest:
        shutil.copyfile(path, os.path.join(directory, 'BEST_' + os.path.basename(path)))
    return path


def load_checkpoint(path, map_location="cpu"):
    """The checkpoint dict (train.py:128), loaded without unpickling code."""
    return torch.load(path, map_location=map_location, weights_only=True)
