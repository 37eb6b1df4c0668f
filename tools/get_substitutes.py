"""Drop-in for CodeXGLUE/Defect-detection/preprocess/get_substitutes.py on the MI355X engine.

Same arguments (--eval_data_file, --base_model, --store_path, --block_size, --index a b) and the
same output (one jsonl line per item with its "substitutes" dict).  --base_model is a local HF
model directory (model.safetensors / pytorch_model.bin, vocab.json + merges.txt) or "synthetic"
(seeded codebert-shaped weights and the repo tokenizer: no checkpoint is reachable offline).
Multi-GPU: launch with torchrun (one rank per GPU); items are pulled from a shared queue and the
shards merged in input order.
"""
import argparse
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _apmc  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eval_data_file", required=True)
    ap.add_argument("--base_model", default="synthetic")
    ap.add_argument("--store_path", required=True)
    ap.add_argument("--block_size", default=512, type=int)
    ap.add_argument("--index", nargs="+", default=["0", "1000000000"])
    ap.add_argument("--precision", default="fp32", choices=["fp32", "f32x3", "bf16"])
    ap.add_argument("--lang", default="c")
    ap.add_argument("--no_cosine", action="store_true",
                    help="GraphCodeBERT preprocessing: keep every top-60 candidate "
                         "(GraphCodeBERT/Defect-detection/preprocess/get_substitutes.py:72-134)")
    args = ap.parse_args()

    import torch

    from apmc_amd.dist import init_from_env, run_sharded_substitutes
    from apmc_amd.engine import Engine
    from apmc_amd.host import Tokenizer
    from apmc_amd.substitutes import SubstituteGenerator
    from apmc_amd.weights import load_checkpoint, synthetic_state_dict

    dist = init_from_env("nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if args.base_model == "synthetic":
        sd, tok = synthetic_state_dict(seed=0, head="none", with_mlm=True), Tokenizer()
    else:
        base = pathlib.Path(args.base_model)
        sd = load_checkpoint(base)
        tok = Tokenizer(base / "vocab.json", base / "merges.txt")
    eng = Engine(sd, head="none", with_mlm=True, precision=args.precision, device=local)
    gen = SubstituteGenerator(eng, tok, block_size=args.block_size, lang=args.lang,
                              cosine=not args.no_cosine)
    t0 = time.time()
    done = [0]

    def progress(idx, item):  # a line a minute or so: long runs stay visibly alive
        done[0] += 1
        if done[0] % 50 == 0:
            print(f"[get_substitutes] {done[0]} items ({idx}) in {time.time() - t0:.0f} s",
                  file=sys.stderr, flush=True)

    tot = run_sharded_substitutes(gen, args.eval_data_file, args.store_path,
                                  int(args.index[0]), int(args.index[1]),
                                  device=torch.device(f"cuda:{local}"), log=progress)
    if dist is None or dist.get_rank() == 0:
        print(f"{tot['items']} items, {tot['occurrences']} occurrences, "
              f"{tot['encoded_seqs']} re-encoded sequences in {time.time() - t0:.1f} s")
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
