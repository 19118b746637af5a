"""Re-tune the C4 decode GEMM shapes (M = 256 greedy / 1280 beam-5 rows) live and write a table.

  python tools/retune_decode.py OLD_TABLE NEW_TABLE
Loads OLD_TABLE minus its decode-shape entries, runs greedy + beam-5 once at B = 256 (each missing
shape is tuned on an idle device, gemm_bf16.hip tune()), and saves every choice to NEW_TABLE."""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
old, new = sys.argv[1], sys.argv[2]
keep = [l for l in open(old) if not (l.startswith("g ") and l.split()[1] in ("256", "1280") and l.split()[4:6] == ["0", "0"])]
tmp = tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False)
tmp.writelines(keep)
tmp.close()
os.environ["CAPGEN_TUNE_TABLE"] = tmp.name
import torch  # noqa: E402

from capgen import _lib, preset  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import reference_init_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402

cfg = preset("C2", dtype="bf16")
dev = torch.device("cuda", 0)
eng = Engine(cfg, dev)
eng.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
eng.set_training(False)
f, p, _ = synthetic_batch(256, 36, cfg.encode_dim_features, cfg.encode_dim_positions, cfg.max_length, cfg.num_vocab,
                          seed=7)
f, p = f.to(dev, torch.bfloat16).contiguous(), p.to(dev).contiguous()
eng.greedy(f, p, want_attention=False)
eng.beam(f, p, 5)
torch.cuda.synchronize()
print("live-tuned shapes:", _lib.tune_live_count(), "saved:", _lib.tune_save(new))
