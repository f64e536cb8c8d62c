import numpy as np, torch, sys
sys.path.insert(0, '.')
from recommender_amd.ctr.model import DLRM
from recommender_amd.sharded import Comm, ShardedSlabEmbedding
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities
DEV = 'cuda'
cards = criteo_cardinalities(200_000, 26)
g = torch.Generator(device=DEV); g.manual_seed(1)
m1 = DLRM([64, 32], [64, 1], 32, sum(cards), 26, 13, device=DEV, slot_cardinalities=cards, generator=g)
emb = ShardedSlabEmbedding(cards, 32, Comm(), device=DEV, full_weight=m1.embedding_layer.weight)
m2 = DLRM([64, 32], [64, 1], 32, sum(cards), 26, 13, device=DEV, embedding_layer=emb)
sd = {k: v for k, v in m1.state_dict().items() if not k.startswith("embedding_layer")}
res = m2.load_state_dict(sd, strict=False)
print("missing", res.missing_keys, "unexpected", res.unexpected_keys)
for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
    print(n1, n2, (p1 - p2).abs().max().item() if p1.shape == p2.shape and p1.numel() else 'skip')
print('table diff', (emb.shard.weight - m1.embedding_layer.weight).abs().max().item())
r = np.random.default_rng(0)
cat, dn, lb = criteo_batch(r, 1024, cards)
b = tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb))
with torch.no_grad():
    x = {"cat_features": b[0], "int_features": b[1]}
    p1 = m1(x); p2 = m2(x)
    print('logit diff nograd', (p1 - p2).abs().max().item())
p1 = m1(x); p2 = m2(x)
print('logit diff grad', (p1 - p2).abs().max().item())
# intermediate: interaction outputs
from recommender_amd.functional import dlrm_interaction
with torch.no_grad():
    bm = m1.bottom_mlp(b[1].float())
    z1 = dlrm_interaction(m1.embedding_layer, b[0], bm, True)
    view, inv = emb.exchange(b[0])
    z2 = dlrm_interaction(view, inv, bm, True)
    print('z diff', (z1 - z2).abs().max().item(), 'U', view.input_dim, 'inv range', inv.min().item(), inv.max().item())
    rows = global_rows = None
    w = m1.embedding_layer.weight
    so = m1.embedding_layer.slot_offsets
    grow = (b[0] + so[:-1][None, :]).reshape(-1)
    print('gathered-by-inverse vs table diff', (view.weight[inv.reshape(-1).long()] - w[grow]).abs().max().item())
from recommender_amd.functional import binary_crossentropy
pa = m1(x); pb = m2(x)
print('manual', float(binary_crossentropy(b[2], pa)), float(binary_crossentropy(b[2], pb)), (pa-pb).abs().max().item())
print('label dtype', b[2].dtype, b[2].shape, pa.shape)
from recommender_amd.ctr.train import TrainStep
s1, s2 = TrainStep(m1, "sgd", lr=0.05), TrainStep(m2, "sgd", lr=0.05)
l1 = s1(b); print('l1', float(l1), float(binary_crossentropy(b[2], m1(x))))
l2 = s2(b); print('l2', float(l2))
