"""BASELINE config C5 on one MI355X: on-GPU RetCCL ResNet-50 tile encoder + TransMIL(2048).

One step = tiles [1, N, 3, 224, 224] (bf16, resident in HBM) -> frozen encoder (train-mode
BatchNorm as the reference runs it under Lightning, or --encoder-mode eval: BN folded into the
convolutions) -> features [1, N, 2048] on the device -> TransMIL(2, 2048) fwd (RCC _fc1 branch,
dropout on) -> CE -> bwd -> Lookahead(RAdam).  Prints one JSON line: slides/sec, ms/step, the
encoder alone (ms, tiles/s, achieved TFLOP/s against the dense bf16 peak), the MIL part alone,
a ``roofline`` object for the encoder (the step's dominant part: library convolutions + the HIP
1x1 / BatchNorm passes) and a ``cpu_baseline``: the fp32 CPU oracle of the same step on a stated
sample (oracle/encoder_ref.py on ``--cpu-tiles`` tiles, extrapolated per tile to N, plus the
TransMIL(2048) oracle fwd + CE + bwd + RAdam step at N measured whole).

    python scripts/bench_c5.py [--n 4096] [--steps 20] [--warmup 3] [--encoder-mode train|eval] [--graph]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BF16_PEAK_TFS = 2500.0
R50_GFLOP_PER_TILE = 4.09   # ResNet-50 forward at 224x224, multiply-adds x 2 (conv + fc-free)


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-tiles", type=int, default=64, help="tiles of the CPU encoder sample (0: no cpu_baseline)")
    ap.add_argument("--encoder-mode", default="train", choices=["train", "eval"])
    # tiles per encoder piece: 1024 measured faster than 512 (eval 84.5 vs 89.0 ms per 4096 tiles;
    # smaller pieces slower: profiles/r04u_c5_chunks.txt); every piece tensor stays < 2 GiB (bf16: the
    # encoder clamps pieces to max_tiles_per_call() = 1337 tiles)
    ap.add_argument("--chunk", type=int, default=1024)
    ap.add_argument("--graph", action="store_true", help="capture the step in a hipGraph")
    ap.add_argument("--layout", default="nhwc", choices=["nhwc", "nchw"])
    # MIOpen find (torch.backends.cudnn.benchmark) picks the 3x3 / stem convolution kernels by timing
    # them once per shape before the timed region: eval encoder 98.9 -> 89.1 ms per 4096 tiles
    # (profiles/r04p_c5_find.jsonl); --no-benchmark keeps MIOpen's immediate-mode heuristics
    ap.add_argument("--benchmark", action=argparse.BooleanOptionalAction, default=True,
                    help="torch.backends.cudnn.benchmark (MIOpen find)")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.benchmark
    from transmil_deepgraft_amd.encoder import ImageBagModel, retccl_resnet50
    from transmil_deepgraft_amd.interface import GradAllReduce, TransMILTask
    from transmil_deepgraft_amd.models import TransMIL
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    enc = retccl_resnet50(chunk=a.chunk).to(dev).set_compute_dtype(torch.bfloat16)
    enc.channels_last = a.layout == "nhwc"
    enc.train(a.encoder_mode == "train")
    mil = TransMIL(2, 2048, 512).to(dev).train()
    model = ImageBagModel(enc, mil)
    task = TransMILTask(mil)
    opt = task.configure_optimizers()[0][0]
    GradAllReduce(mil.parameters(), model=mil)        # gradient bucket (no-op collective at N = 1)
    g = torch.Generator(device=dev).manual_seed(7)
    tiles = torch.randn(1, a.n, 3, 224, 224, device=dev, generator=g).to(torch.bfloat16)
    label = torch.tensor([1], device=dev)

    def step():
        logits = model(tiles)
        loss = task.loss(logits, torch.nn.functional.one_hot(label, 2).float())
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(a.warmup):
        step()
    run = step
    if a.graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        run = graph.replay
    t_step = timed(run, a.steps)
    with torch.no_grad():
        t_enc = timed(lambda: enc(tiles[0]), a.steps)
        feats = enc(tiles[0])[None]

    def mil_step():
        loss = task.loss(mil(feats), torch.nn.functional.one_hot(label, 2).float())
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    t_mil = timed(mil_step, a.steps)
    enc_tfs = R50_GFLOP_PER_TILE * a.n / t_enc / 1e3
    cpu = cpu_baseline(a, enc, mil) if a.cpu_tiles > 0 else None
    print(json.dumps({
        "metric": f"slides/sec (fwd+bwd) end-to-end, RetCCL ResNet-50 encoder + TransMIL(2048), N={a.n} tiles",
        "value": round(1.0 / t_step, 3), "unit": "slides/sec", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(t_step * 1e3, 3), "higher_is_better": True, "dtype": "bf16",
        "data": "synthetic (randn tiles resident in HBM, random-init weights)",
        "config": {"workload": f"C5: 1 slide x {a.n} tiles 3x224x224 -> ResNet-50 (frozen, BN "
                               f"{'batch stats' if a.encoder_mode == 'train' else 'folded'}) -> TransMIL 2-class",
                   "execution": "hipGraph" if a.graph else "eager", "chunk": a.chunk, "layout": a.layout,
                   "miopen_find": a.benchmark},
        "encoder": {"ms": round(t_enc * 1e3, 3), "tiles_per_s": round(a.n / t_enc, 1),
                    "achieved_tfs": round(enc_tfs, 1), "peak_tfs": BF16_PEAK_TFS,
                    "frac": round(enc_tfs / BF16_PEAK_TFS, 4), "mode": a.encoder_mode,
                    "flops_note": f"{R50_GFLOP_PER_TILE} GFLOP per 224x224 tile (ResNet-50 forward)"},
        "mil_ms": round(t_mil * 1e3, 3),
        "roofline": {"bound": "mfma", "achieved": round(enc_tfs, 1), "peak": BF16_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": round(enc_tfs / BF16_PEAK_TFS, 4), "traffic": None,
                     "kernel": f"encoder ({a.encoder_mode} BN): hand-written stem (conv + BN + ReLU + pool, "
                               "tm_stem_*), MIOpen / CK 3x3 convolutions, hipBLASLt 1x1 GEMMs (tm_conv1x1), "
                               "HIP BatchNorm / bias passes",
                     "algorithmic_flops": int(R50_GFLOP_PER_TILE * 1e9 * a.n), "ms": round(t_enc * 1e3, 3)},
        "cpu_baseline": cpu,
    }), flush=True)


def cpu_baseline(a, enc, mil):
    """The same step on the host's cores through the fp32 oracles: the encoder on a --cpu-tiles sample
    (oracle/encoder_ref.py, the mode's BatchNorm: train = that sample's batch statistics), median of 3,
    scaled per tile to N; the TransMIL(2048) oracle (oracle/transmil_ref.py) fwd + CE + bwd + RAdam at
    N features, median of 3 after one warm-up.  Slides/s = 1 / (extrapolated encoder + MIL step)."""
    import statistics
    from oracle.encoder_ref import features
    from oracle.transmil_ref import TransMIL as RefTransMIL
    threads = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    torch.set_num_threads(threads)
    sd = {k: v.detach().float().cpu() for k, v in enc.state_dict().items()}
    g = torch.Generator().manual_seed(11)
    x = torch.randn(a.cpu_tiles, 3, 224, 224, generator=g)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        features(x, sd, dtype=torch.float32, train=a.encoder_mode == "train")
        ts.append(time.perf_counter() - t0)
    t_tile = statistics.median(ts) / a.cpu_tiles
    torch.manual_seed(0)
    ref = RefTransMIL(2, 2048, 512).train()
    opt = torch.optim.RAdam(ref.parameters(), lr=2e-4)
    feats = torch.rand(1, a.n, 2048)
    y = torch.nn.functional.one_hot(torch.tensor([1]), 2).float()

    def step():
        loss = torch.nn.functional.cross_entropy(ref(feats), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    step()
    ms = []
    for _ in range(3):
        t0 = time.perf_counter()
        step()
        ms.append(time.perf_counter() - t0)
    t_mil = statistics.median(ms)
    t_slide = t_tile * a.n + t_mil
    return {"value": round(1.0 / t_slide, 5), "unit": "slides/sec", "cores": threads, "kind": "port",
            "sample": f"encoder: oracle/encoder_ref.py fp32 on {a.cpu_tiles} tiles ({a.encoder_mode} BN), median of 3, "
                      f"{t_tile * 1e3:.1f} ms per tile extrapolated x {a.n} tiles (EXTRAPOLATED); TransMIL(2048) oracle "
                      f"fwd+CE+bwd+RAdam at N={a.n} measured, median of 3: {t_mil:.3f} s",
            "encoder_s_per_tile": round(t_tile, 5), "mil_step_s": round(t_mil, 4)}


if __name__ == "__main__":
    main()
