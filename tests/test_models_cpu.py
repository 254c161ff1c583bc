"""Model families beyond the reference CNN (BASELINE.json stretch configs): shapes, parameter
counts and one CPU forward/backward each."""
import torch

from mihvd.models.bert import BertConfig, BertForMaskedLM, synthetic_mlm_batch
from mihvd.models.resnet import ResNet50, num_params


def test_resnet50_shape_and_params():
    m = ResNet50()
    assert num_params(m) == 25_557_032  # torchvision's resnet50 count
    x = torch.randn(2, 3, 64, 64)
    out = m(x)
    assert out.shape == (2, 1000)
    out.sum().backward()
    assert all(p.grad is not None for p in m.parameters())


def test_bert_base_params_and_small_step():
    big = BertForMaskedLM(BertConfig())
    n = sum(p.numel() for p in big.parameters())
    assert 109_000_000 < n < 111_000_000  # BERT-base MLM with tied decoder
    c = BertConfig(vocab_size=101, hidden=32, layers=2, heads=4, ffn=64, max_len=16)
    m = BertForMaskedLM(c)
    ids, labels = synthetic_mlm_batch(2, 16, c.vocab_size, "cpu", mask_prob=0.5)
    ids = ids.clamp_max(c.vocab_size - 1)
    loss = m(ids, labels)
    loss.backward()
    assert torch.isfinite(loss) and m.tok.weight.grad is not None
