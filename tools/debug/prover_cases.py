import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
import dusk_plonk_amd as plk
from dusk_plonk_amd.prover import PlonkKey, Constraint, fr_int
from oracle_lib import random_fr
from verifier import verify, VerificationError

tau_l = random_fr(1, seed=7)[0]; tau = fr_int(tau_l)
pp = plk.PlonkParams.setup(6, tau_l)

class C:
    def __init__(self, pub, extra, a=10, b=20):
        self.pub, self.extra, self.a, self.b = pub, extra, a, b
    def synthesize(self, cs):
        wa, wb = cs.append_witness(self.a), cs.append_witness(self.b)
        wc = cs.gate_add(Constraint().left(1).right(1).a(wa).b(wb))
        if self.pub:
            cs.assert_equal_constant(wc, 0, -(self.a + self.b))
        else:
            cs.assert_equal_constant(wc, self.a + self.b)
        for _ in range(self.extra):
            w = cs.append_witness(1); cs.component_boolean(w)

for pub in (False, True):
    for extra in (0, 1, 9):
        prover, vd = PlonkKey.compile_with_circuit(pp, b"t", C(pub, extra, 2, 3) if pub else C(pub, extra))
        proof, pi = prover.create_proof(5, C(pub, extra))
        try:
            verify(vd, proof, pi, tau); res = "OK"
        except VerificationError as e:
            res = "FAIL"
        print(f"pub={pub} extra={extra} m={vd.m} n={vd.n} pi={pi} -> {res}", flush=True)
