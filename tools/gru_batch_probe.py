"""Largest mission-GRU batch MIOpen's RNN accepts (Embedding(32,32) -> GRU(32,128), 128 tokens),
forward with and without autograd, plus backward.  Prints one line per batch size."""
import torch
from torch import nn

torch.manual_seed(0)
emb = nn.Embedding(32, 32).cuda()
gru = nn.GRU(32, 128, 1, True, True).cuda()
for B in (2048, 4096, 6144, 8192, 12288, 16384, 24576, 32768):
    tok = torch.randint(0, 32, (B, 128), device="cuda")
    res = []
    for mode in ("nograd", "grad"):
        try:
            if mode == "nograd":
                with torch.no_grad():
                    _, h = gru(emb(tok))
            else:
                _, h = gru(emb(tok))
                h.sum().backward()
            torch.cuda.synchronize()
            res.append("%s ok" % mode)
        except RuntimeError as e:
            res.append("%s FAIL(%s)" % (mode, str(e)[:40]))
    print(B, " | ".join(res), flush=True)
