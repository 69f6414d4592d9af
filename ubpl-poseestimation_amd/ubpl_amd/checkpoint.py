"""Model selection and checkpoint payloads of the epoch loop
(projects/MT_UBPL.py:86-103, projects/DualPose_UBPL.py:83-100), in the
reference's key schema, so a checkpoint written here loads into the
reference's models / torch.optim.AdamW and the other way round.

The file itself is written by the reference's own CommUtils.ckpt_save
(utils/base/comm.py:92-103: torch.save to <ckptPath>/checkpoint.pth.tar, copied
to checkpoint_best.pth.tar when is_best); save_checkpoint below does the same
for callers without the reference tree.  Loading uses torch.load(...,
weights_only=True): a checkpoint is tensors, numbers and lists only.
"""
import os
import shutil

import torch


def select_best(accs_arrays, args, epo):
    """projects/MT_UBPL.py:88-95: per entry (each teacher, then their mean),
    best if its mean PCK (last element) beats args.best_acc[idx]; updates
    args.best_acc / args.best_epoch in place.  Returns the is_best list."""
    is_best = []
    for idx in range(len(args.best_epoch)):
        flag = accs_arrays[idx][-1] > args.best_acc[idx]
        is_best.append(flag)
        if flag:
            args.best_epoch[idx] = epo
            args.best_acc[idx] = accs_arrays[idx][-1]
    return is_best


def checkpoint_state(models, models_ema, optims, args, epo):
    """projects/MT_UBPL.py:97-101: {current_epoch, best_acc, best_epoch,
    model<b>_state, model<b>_ema_state, optim<b>_state} for b = 1..brNum."""
    ck = {"current_epoch": epo, "best_acc": args.best_acc, "best_epoch": args.best_epoch}
    for b in range(len(models)):
        ck["model{}_state".format(b + 1)] = models[b].state_dict()
        ck["model{}_ema_state".format(b + 1)] = models_ema[b].state_dict()
        ck["optim{}_state".format(b + 1)] = optims[b].state_dict()
    return ck


def save_checkpoint(state, is_best, ckpt_path="ckpts"):
    """utils/base/comm.py:92-103 (same file names, same best-copy rule)."""
    os.makedirs(ckpt_path, exist_ok=True)
    path = os.path.join(ckpt_path, "checkpoint.pth.tar")
    torch.save(state, path)
    if is_best:
        shutil.copyfile(path, os.path.join(ckpt_path, "checkpoint_best.pth.tar"))
    return path


def load_checkpoint(path, models, models_ema, optims, map_location=None):
    """Restore a checkpoint of the schema above (ours or the reference's):
    models, teachers (parameters and BN buffers) and optimiser states.
    Returns (current_epoch, best_acc, best_epoch)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    for b in range(len(models)):
        models[b].load_state_dict(ck["model{}_state".format(b + 1)])
        models_ema[b].load_state_dict(ck["model{}_ema_state".format(b + 1)])
        optims[b].load_state_dict(ck["optim{}_state".format(b + 1)])
    return ck["current_epoch"], ck["best_acc"], ck["best_epoch"]
