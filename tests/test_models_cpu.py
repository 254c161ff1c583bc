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


def test_bert_gather_embeddings_match_embedding_lookups():
    """BertConfig.embedding_impl="gather" (index_select lookups: an index_add_ backward that replays
    from a HIP graph) computes the same loss and gradients as F.embedding's lookups."""
    import torch

    from mihvd.models.bert import BertConfig, BertForMaskedLM

    torch.manual_seed(0)
    m = BertForMaskedLM(BertConfig(hidden=64, layers=1, heads=4, ffn=128, max_len=32, vocab_size=100)).eval()
    ids = torch.randint(0, 100, (2, 16))
    ids[:, ::3] = 7  # repeated ids, as [MASK] tokens are
    labels = torch.where(torch.rand(2, 16) < 0.5, ids, torch.full_like(ids, -100))
    out = []
    for impl in ("gather", "embedding"):
        m.c.embedding_impl = impl
        m.zero_grad()
        loss = m(ids, labels)
        loss.backward()
        out.append((loss.detach(), [p.grad.clone() for p in m.parameters()]))
    assert torch.allclose(out[0][0], out[1][0], rtol=0, atol=1e-6)
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
