"""Seeded initial parameters of the NS model: mag.REGNN / mag.REGCNConv
consume the RNG stream in the reference's order -- every module constructed, then
REGNN.reset_parameters() again (mag/regnn_ns.py:247-298), REGCNConv drawing weight_root (= weight)
a second time when residual (mag/regnn_layers.py:71-78) -- so torch.manual_seed(s) gives the
reference's initial weights bit for bit. Fixture: tests/golden/make_golden.py gen_regnn_init (the
reference's REGNN class, float32)."""
import numpy as np
import pytest
import torch

import os

import _golden as G

if not os.path.exists(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                   "mag_regnn_init.npz")):
    pytest.skip("fixture tests/golden/mag_regnn_init.npz absent", allow_module_level=True)
D = G.load("mag_regnn_init")


@pytest.mark.parametrize("i", range(len(D["meta"]["configs"])))
def test_regnn_seeded_init_matches_reference(i):
    from regnn_hip import mag
    c = D["meta"]["configs"][i]
    counts = {t: n for t, n in enumerate(c["counts"])}
    torch.manual_seed(c["seed"])
    m = mag.REGNN(c["in_channels"], c["hidden"], c["classes"], c["num_layers"],
                  c["scaling_factor"], c["dropout"], {t: c["dims"][t] for t in range(4)},
                  c["num_edge_types"], residual=c["residual"], use_norm="ln", self_loop_type=2,
                  feats_type=c["feats_type"], num_nodes_dict=counts,
                  target_node_type=c["target_type"])
    want = G.sub(D, f"c{i}_p_", np.float32)
    got = {n: p.detach().numpy() for n, p in m.named_parameters()}
    assert set(got) == set(want)
    for n, v in want.items():
        assert np.array_equal(got[n], v), n
