"""Child of tests/kernels/test_stream_check_gpu.py (also runnable by hand to read the full
race report): two training steps (selective recompute, grad accumulation 2) under the
torch.cuda stream sanitizer."""
import torch

from llmctl.runtime.engine import TrainingConfig, TrainingEngine

cfg = TrainingConfig(model_name_or_path="tiny", device="cuda", seq_len=128, batch_size=2, log_level="error",
                     activation_checkpoint="selective", gradient_accumulation_steps=2, output_dir="/tmp/sc")
eng = TrainingEngine(cfg)
g = torch.Generator(device="cuda").manual_seed(0)
for s in range(2):
    b = [(torch.randint(1, 500, (2, 128), device="cuda", generator=g),
          torch.randint(1, 500, (2, 128), device="cuda", generator=g)) for _ in range(2)]
    out = eng.train_step(b)
torch.cuda.synchronize()
print("loss", float(out["loss"]))
