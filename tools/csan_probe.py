"""GPU-box: PyTorch's CUDA sanitizer (CSAN) over the eager MT_UBPL step with
per-network streams.

CSAN sees every dispatcher op — torch's own and the ubpl torch ops, whose
schemas mark each mutable pointer `Tensor(a!)` — and checks that every pair
of accesses to one tensor from two streams is ordered by stream order or a
recorded event wait (not by timing), so a missing cross-stream dependency
shows up even where eager host pacing hides it.

Stock CSAN keys tensors by data pointer (two views of one flat buffer at
different offsets are distinct to it) and stops at the first race.  With
`storage` it keys them by their storage's base pointer instead (every view of
a buffer is one tensor: no missed overlaps, possible false positives between
disjoint views), and with `all` it records every race and goes on, printing
one line per distinct (op, stream pair, source line).

usage: python tools/csan_probe.py [case] [steps] [storage] [all]
"""
import collections
import contextlib
import io
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402
import torch.cuda._sanitizer as csan  # noqa: E402

FOUND = collections.Counter()


def _where(stack):
    fr = [f for f in (stack or []) if "ubpl_amd" in f.filename or "/tools/" in f.filename]
    return " <- ".join("%s:%d" % (os.path.basename(f.filename), f.lineno) for f in fr[-3:][::-1]) or "?"


def _patch(storage, keep_going):
    if storage:
        def _h(self, value, is_write, metadata_only, name=None, is_output=False):
            if isinstance(value, torch.Tensor) and value.is_cuda:
                dp = value.untyped_storage().data_ptr()
                if is_write:
                    self.dataptrs_written.add(dp)
                elif not metadata_only:
                    self.dataptrs_read.add(dp)
                self.tensor_aliases.setdefault(dp, [])
                if name is not None:
                    self.tensor_aliases[dp].append(name)
                if is_output:
                    self.outputs.add(dp)
        csan.ArgumentHandler._handle_argument = _h
    if keep_going:
        def disp(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            is_factory = bool(csan.FACTORY_FUNCTION_REGEX.match(func._schema.name))
            ah = csan.ArgumentHandler()
            ah.parse_inputs(func._schema, args, kwargs, is_factory=is_factory)
            out = func(*args, **kwargs)
            ah.parse_outputs(func._schema, out, is_factory=is_factory)
            errs = self.event_handler._handle_kernel_launch(
                torch.cuda.current_stream().cuda_stream, ah.dataptrs_read - ah.dataptrs_written,
                ah.dataptrs_written, ah.outputs, func._schema, ah.tensor_aliases)
            for e in errs or []:
                cur = traceback.extract_stack()
                prev = e.previous_access
                FOUND[("%s [%s]" % (func._schema.name, _where(cur)),
                       "prev %s [%s]" % (prev.operator.split("(")[0] if prev else "-",
                                        _where(prev.stack_trace) if prev else "-"))] += 1
            return out
        csan.CUDASanitizerDispatchMode.__torch_dispatch__ = disp


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "mt_ubpl"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    storage = "storage" in sys.argv[3:]
    keep_going = "all" in sys.argv[3:]
    os.environ["UBPL_STEP_GRAPH"] = "0"
    import seeds
    from oracle import render as OR
    from ubpl_amd import train as T
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW

    # The autograd engine makes a node's stream wait for the streams its input
    # gradients were produced on with c10 events that do not reach CSAN's
    # trace hooks; restate that wait (the network gradients come from the
    # loss backward on the default stream) so CSAN sees it.
    import ubpl_amd.hourglass as HG
    _bwd = HG._HourglassFn.backward

    def _bwd_seen(ctx, dpreds, dfeats):
        torch.cuda.current_stream().wait_stream(torch.cuda.default_stream())
        return _bwd(ctx, dpreds, dfeats)
    HG._HourglassFn.backward = staticmethod(_bwd_seen)

    cfg = seeds.step_cases()[case]
    models, emas, _ = seeds.step_models(lambda k, s, m: StackedHourglass(k, s, m), cfg, device="cuda")
    optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    batches = list(loader) * steps
    torch.cuda.synchronize()
    _patch(storage, keep_going)
    csan.enable_cuda_sanitizer()
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            T.train_mt_ubpl(batches, models, emas, optims, args)
        torch.cuda.synchronize()
    except csan.CUDASanitizerErrors as e:
        print("CSAN: %d error(s)" % len(e.errors), flush=True)
        for err in e.errors[:4]:
            print(str(err)[:6000], flush=True)
        sys.exit(3)
    mode = "storage" if storage else "data pointer"
    if not FOUND:
        print("CSAN (%s keys): no unsynchronized cross-stream access in %d step(s) of %s" % (mode, steps, case),
              flush=True)
        return
    print("CSAN (%s keys): %d distinct race sites, %d accesses" % (mode, len(FOUND), sum(FOUND.values())))
    for (cur, prev), n in FOUND.most_common(60):
        print("%5d  %s\n       %s" % (n, cur, prev))


if __name__ == "__main__":
    main()
