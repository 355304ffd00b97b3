import sys, numpy as np
sys.path[:0] = ['.', 'oracle']
import snake_amd as snk, oracle
m = snk.DQNModel(12, 3, n_frames=2, seed=5)
rng = np.random.default_rng(1)
P = m.P
g = (rng.standard_normal(P) * 10.0 ** rng.uniform(-9, 0, P)).astype(np.float32)
acc = (np.abs(rng.standard_normal(P)) * 1e-3).astype(np.float32)
acc[::7] = 0
th = m.get_params()
m.set_params(g, snk.SNK_NET_GRAD); m.set_params(acc, snk.SNK_NET_OPT_STATE)
m.apply_grad()
th2, acc2 = oracle.rmsprop(th, acc, g)
d_th = m.get_params(); d_acc = m.get_params(snk.SNK_NET_OPT_STATE)
bad_acc = np.nonzero(d_acc != acc2)[0]; bad_th = np.nonzero(d_th != th2)[0]
print("acc mismatches", len(bad_acc), "theta mismatches", len(bad_th))
for i in bad_th[:8]:
    q = acc2[i]
    print(i, "g", g[i], "acc0", acc[i], "q dev/ref", d_acc[i], q, "th dev/ref", d_th[i], th2[i], "upd ref", np.float32(g[i]*np.float32(5e-4))/np.float32(np.sqrt(q)+np.float32(1e-8)))
