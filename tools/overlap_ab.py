"""A/B: C3 clip steps on one stream vs alternating over S streams.

With S > 1, step k runs on stream k % S (its own workspace and label
buffer), so clip k + 1's MFCC launch can start on the CUs clip k's MFCC
tail frees, and clip k's FFN overlaps clip k + 1's MFCC ramp.  Prints
ms/step for S = 1, 2, 3, alternating, three rounds.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    F = 1_000_000
    pipe = VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3)))
    audio = synth_audio(160 * (F - 1) + 401, 100, dev)
    ref = torch.empty((F - 5,), dtype=torch.uint8, device=dev)
    pipe.labels(audio, out=ref)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(2)]
    labs = [torch.empty_like(ref) for _ in streams]
    done = [torch.cuda.Event() for _ in streams]

    def run(S, steps):
        for k in range(steps):
            s = streams[k % S]
            pipe.labels(audio, out=labs[k % S], stream=s)
        torch.cuda.synchronize()

    for S in (1, 2, 3):  # warm-up (workspaces, clocks)
        run(S, 200)
    steps = 200
    for rnd in range(3):
        for S in (1, 2, 3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(S, steps)
            el = time.perf_counter() - t0
            ok = all(torch.equal(l, ref) for l in labs[:S])
            print(f"round {rnd} S={S}: {el * 1e3 / steps:.4f} ms/step labels_ok={ok}", flush=True)
    del done


if __name__ == "__main__":
    main()
