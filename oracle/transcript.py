"""Restatement of the reference verifier's transcript, DEEP (quotiening) and FRI query checks --
TEST INFRASTRUCTURE (the checker), never product code.

It replays, over the data of the reference's own proof.json / vk.json
(tests/golden/proof_fri.json), exactly what Verifier::verify does with it
(cs/implementations/verifier.rs:888-2523) apart from the constraint evaluation at z:

  * the Poseidon2 transcript GoldilocksPoisedon2Transcript
    (AlgebraicSpongeBasedTranscript<GoldilocksField, 8, 12, 4, Poseidon2Goldilocks,
    AbsorptionModeOverwrite>, transcript.rs:48-141) over the sponge's absorb / finalize /
    run_round_function / try_get_commitment (algebraic_props/sponge.rs:241-323);
  * the challenge order of the verifier (verifier.rs:924-1076, 1819-1984) and the FRI schedule
    (compute_fri_schedule, prover.rs:2281-2372);
  * the query indices from BoolsBuffer::get_bits (transcript.rs:369-417): 64 - max_needed
    least significant bits per challenge, inner index = low log n bits, coset = the rest
    (verifier.rs:2050-2068);
  * the domain point x = 7 * prod_i w_{2^(i+1)}^{bit_i} = 7 * w_{nD}^{bitrev(idx)}
    (verifier.rs:2158-2196), the DEEP combination of every base oracle's leaf values at x
    (quotening_operation, verifier.rs:2526-2565, sources in the order of :2226-2390);
  * each FRI step's fold of its leaf (verifier.rs:2396-2488) and the final Horner evaluation of
    final_fri_monomials (:2490-2518).

The permutation is the C oracle's (oracle/boojum_oracle.c, pinned to proof.json's Merkle paths).
Pure-Python integers for the GoldilocksExt2 arithmetic (u^2 = 7, field/goldilocks/extension.rs:4-41).
"""
import numpy as np

import oracle as O

P = 0xFFFFFFFF00000001
GEN = 7            # multiplicative generator (goldilocks/mod.rs:107-114)
NON_RESIDUE = 7    # GoldilocksExt2 (extension.rs:14-16)


# ------------------------------------------------------------------ GoldilocksExt2
def e_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def e_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def e_mul(a, b):
    return ((a[0] * b[0] + NON_RESIDUE * a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def e_mul_base(a, k):
    return (a[0] * k % P, a[1] * k % P)


def e_inv(a):
    # (a0 - a1 u) / (a0^2 - 7 a1^2)
    norm = (a[0] * a[0] - NON_RESIDUE * a[1] * a[1]) % P
    ni = pow(norm, P - 2, P)
    return (a[0] * ni % P, (-a[1]) * ni % P)


def domain_generator(log_n):
    return int(O.domain_generator(log_n)) % P


# ------------------------------------------------------------------ transcript
class Poseidon2Transcript:
    """AlgebraicSpongeBasedTranscript (transcript.rs:48-141) over GoldilocksPoseidon2Sponge with
    AbsorptionModeOverwrite, AW = 8, SW = 12, CW = 4.  The sponge state persists across
    challenges; absorb only ever sees whole 8-element chunks here (the transcript pads)."""

    AW = 8

    def __init__(self):
        self.buffer = []
        self.available = []
        self.state = [0] * 12

    def _permute(self):
        self.state = [int(x) for x in O.poseidon2_permutation(np.array(self.state, dtype=np.uint64))]

    def witness_field_elements(self, els):
        self.buffer.extend(int(e) % P for e in els)

    def witness_merkle_tree_cap(self, cap):
        for d in cap:
            self.witness_field_elements(d)

    def get_challenge(self):
        if not self.buffer:
            if self.available:
                return self.available.pop(0)
            # run_round_function + try_get_commitment::<AW> (sponge.rs:287-298)
            self._permute()
            self.available = self.state[:self.AW]
            return self.get_challenge()
        to_absorb = self.buffer + [1]  # rescue-prime padding
        self.buffer = []
        mult = -(-len(to_absorb) // self.AW)
        to_absorb += [0] * (mult * self.AW - len(to_absorb))
        for i in range(0, len(to_absorb), self.AW):
            # absorb of a whole chunk with filled == 0: overwrite state[..AW], permute (:241-283)
            self.state[:self.AW] = to_absorb[i:i + self.AW]
            self._permute()
        # finalize::<AW> with nothing pending: the commitment state[..AW] (:300-323)
        self.available = self.state[:self.AW]
        return self.get_challenge()

    def get_challenges(self, n):
        return [self.get_challenge() for _ in range(n)]


class BoolsBuffer:
    """transcript.rs:369-417, algebraic branch."""

    def __init__(self, max_needed):
        self.available = []
        self.max_needed = max_needed

    def get_bits(self, transcript, num_bits):
        while len(self.available) < num_bits:
            el = transcript.get_challenge() % P          # as_u64_reduced
            self.available += [bool((el >> i) & 1) for i in range(64 - self.max_needed)]
        out, self.available = self.available[:num_bits], self.available[num_bits:]
        return out


def u64_from_lsb_first_bits(bits):
    return sum(int(b) << i for i, b in enumerate(bits))


def compute_fri_schedule(security_bits, cap_size, pow_bits, rate_log_two, initial_degree_log_two):
    """prover.rs:2281-2372 -> (new_pow_bits, num_queries, schedule, final_degree)."""
    raw = security_bits - pow_bits
    new_pow = pow_bits
    if raw % rate_log_two != 0 and new_pow >= rate_log_two - (raw % rate_log_two):
        new_pow -= rate_log_two - (raw % rate_log_two)
    raw = security_bits - new_pow
    num_queries = raw // rate_log_two + (1 if raw % rate_log_two else 0)
    stop = max(1, cap_size >> rate_log_two)
    stop_log = stop.bit_length() - 1
    deg = initial_degree_log_two
    cap_log = cap_size.bit_length() - 1
    schedule = []
    while deg > stop_log:
        if deg + rate_log_two <= cap_log:
            break
        if deg - stop_log >= 3:
            deg -= 3
            schedule.append(3)
        elif deg - stop_log == 2:
            deg -= 2
            schedule.append(2)
        else:
            deg -= 1
            schedule.append(1)
            break
        if deg + rate_log_two <= cap_log:
            break
    return new_pow, num_queries, schedule, 1 << deg


def materialize_ext_challenge_powers(c, n):
    """prover.rs:2374-2395: [1, c, c^2, ...] in GoldilocksExt2."""
    out = [(1, 0), c]
    cur = c
    for _ in range(2, n):
        cur = e_mul(cur, c)
        out.append(cur)
    return out[:n]


# ------------------------------------------------------------------ circuit geometry
def geometries(fx):
    """The verifier's size calculators (verifier.rs:655-887) for proof.json's circuit.  The
    specialised-column counts (variables / witnesses / constants the circuit's gates place in
    specialised columns) are not in the VK; the four base-oracle leaf sizes and values_at_z's
    length leave a few candidates, and only one of them passes the DEEP check (replay tries them
    in turn).  Yields dicts V, W, C, M, L, I, lookup_setups, quotient_degree."""
    vk = fx["vk"]
    par = vk["parameters"]
    lp = vk["lookup_parameters"]
    kind, lpar = next(iter(lp.items()))
    assert kind == "UseSpecializedColumnsWithTableIdAsConstant", kind
    n = vk["domain_size"]
    q0 = fx["queries"][0]
    leaf = {k: len(q0[k + "_query"]["leaf_elements"]) for k in ("witness", "stage_2", "quotient", "setup")}
    L = lpar["num_repetitions"]                                 # num_sublookup_arguments
    M = -(-vk["total_tables_len"] // n)                         # num_multipicities_polys
    lookup_setups = lpar["width"] + 1                           # num_lookup_table_setup_polys
    qd = vk["quotient_degree"]
    # stage 2 = 2 (1 + I + L + M); I = num_intermediate_partial_product_relations(V, qd)
    I = leaf["stage_2"] // 2 - 1 - L - M
    assert leaf["quotient"] == 2 * qd
    assert 1 == len(fx["values_at_z_omega"]) and L + M == len(fx["values_at_0"])
    found = False
    for V in range(par["num_columns_under_copy_permutation"], leaf["witness"] + 1):
        if V <= qd or -(-V // qd) - 1 != I:
            continue
        W = leaf["witness"] - V - M
        C = leaf["setup"] - V - lookup_setups
        if W < par["num_witness_columns"] or C < par["num_constant_columns"] + vk["extra_constant_polys_for_selectors"]:
            continue
        g = dict(V=V, W=W, C=C, M=M, L=L, I=I, lookup_setups=lookup_setups, quotient_degree=qd)
        n_at_z = V + W + C + V + 1 + I + M + L + M + lookup_setups + qd
        if n_at_z == len(fx["values_at_z"]):
            found = True
            yield g
    assert found, "no geometry matches the leaf sizes"


# ------------------------------------------------------------------ the replay
def replay(fx):
    """Replays the verifier over the fixture under the one circuit geometry that verifies (see
    geometries).  Returns a dict with the challenges, the FRI schedule, the geometry and, per
    query, its index, its x, the DEEP value and each FRI step's (leaf value, folded value);
    AssertionError if no geometry passes, with the first candidate's failure."""
    first = None
    for g in geometries(fx):
        try:
            return replay_with(fx, g)
        except AssertionError as e:
            first = first or e
    raise first


def replay_with(fx, g, x_convention="bitrev"):
    """The verifier's checks (see module doc) under circuit geometry g.  x_convention "natural"
    (x = 7 w^idx instead of 7 w^bitrev(idx)) exists only for the negative test that shows the
    DEEP check pins the LDE domain convention."""
    vk = fx["vk"]
    cfg = fx["proof_config"]
    n = vk["domain_size"]
    log_n = n.bit_length() - 1
    lde_factor = cfg["fri_lde_factor"]
    cap_size = cfg["merkle_tree_cap_size"]
    tr = Poseidon2Transcript()
    tr.witness_merkle_tree_cap(vk["setup_merkle_tree_cap"])                   # :924
    for v in fx["public_inputs"]:                                             # :944
        tr.witness_field_elements([v])
    tr.witness_merkle_tree_cap(fx["witness_oracle_cap"])                      # :952
    beta, gamma = tr.get_challenges(2), tr.get_challenges(2)                  # :955-957
    lookup_beta, lookup_gamma = tr.get_challenges(2), tr.get_challenges(2)    # :962-964
    tr.witness_merkle_tree_cap(fx["stage_2_oracle_cap"])                      # :978
    alpha = tr.get_challenges(2)                                              # :981
    tr.witness_merkle_tree_cap(fx["quotient_oracle_cap"])                     # :1059
    z = tuple(tr.get_challenges(2))                                           # :1063
    for s in ("values_at_z", "values_at_z_omega", "values_at_0"):             # :1067-1077
        for v in fx[s]:
            tr.witness_field_elements(v)
    # public inputs grouped by opening point w^row (:1080-1110)
    omega = domain_generator(log_n)
    pi_tuples = []
    for (col, row), val in zip(vk["public_inputs_locations"], fx["public_inputs"]):
        at = pow(omega, row, P)
        for t in pi_tuples:
            if t[0] == at:
                t[1].append((col, val))
                break
        else:
            pi_tuples.append((at, [(col, val)]))
    c = tuple(tr.get_challenges(2))                                           # :1819-1820
    total = len(fx["values_at_z"]) + len(fx["values_at_z_omega"]) + len(fx["values_at_0"]) + \
        sum(len(s) for _, s in pi_tuples)
    deep_ch = materialize_ext_challenge_powers(c, total)
    new_pow, num_queries, schedule, final_degree = compute_fri_schedule(
        cfg["security_level"], cap_size, cfg["pow_bits"], lde_factor.bit_length() - 1, log_n)
    assert new_pow == cfg["pow_bits"]
    fri_ch = []
    caps = [fx["fri_base_oracle_cap"]] + fx["fri_intermediate_oracles_caps"]
    assert len(caps) == len(schedule)
    for cap, d in zip(caps, schedule):                                        # :1858-1927
        tr.witness_merkle_tree_cap(cap)
        ch = tuple(tr.get_challenges(2))
        powers = [ch]
        for _ in range(1, d):
            powers.append(e_mul(powers[-1], powers[-1]))
        fri_ch.append(powers)
    mono = fx["final_fri_monomials"]
    assert len(mono[0]) == final_degree == len(mono[1])
    tr.witness_field_elements(mono[0])                                        # :1954-1955
    tr.witness_field_elements(mono[1])
    assert cfg["pow_bits"] == 0   # no PoW challenges drawn (:1957-1984)

    lde_size = n * lde_factor
    max_needed = lde_size.bit_length() - 1
    bools = BoolsBuffer(max_needed)
    inner_bits = log_n
    pw = [domain_generator(i) for i in range(max_needed + 1)]
    pw_inv = [pow(x, P - 2, P) for x in pw]
    w4i, w8i = pw_inv[2], pw_inv[3]
    interpolation_steps = [1, w4i, w8i, w4i * w8i % P]                        # :2031-2043
    V, W, C, M, L, I = (g[k] for k in ("V", "W", "C", "M", "L", "I"))
    out_queries = []
    for q in fx["queries"]:
        bits = bools.get_bits(tr, max_needed)                                 # :2051-2068
        inner = u64_from_lsb_first_bits(bits[:inner_bits])
        coset = u64_from_lsb_first_bits(bits[inner_bits:])
        idx = (coset << log_n) + inner
        for name, cap in (("witness", fx["witness_oracle_cap"]), ("stage_2", fx["stage_2_oracle_cap"]),
                          ("quotient", fx["quotient_oracle_cap"]), ("setup", vk["setup_merkle_tree_cap"])):
            qq = q[name + "_query"]
            assert O.verify_proof_over_cap(qq["proof"], cap, O.hash_into_leaf(qq["leaf_elements"]), idx), \
                "%s query not in tree at %d" % (name, idx)
        x = 1
        for b, wp in zip(bits, pw[1:]):                                       # :2162-2171
            if b:
                x = x * wp % P
        if x_convention == "natural":
            x = pow(pw[max_needed], idx, P)
        power_chunks, skip = [], 0                                            # :2173-2190
        for d in schedule:
            e = 1
            for j, (b, wi) in enumerate(zip(bits[skip:], pw_inv[1:])):
                if j >= d and b:
                    e = e * wi % P
            skip += d
            power_chunks.append(e)
        xq = x * GEN % P
        wl, sl = q["witness_query"]["leaf_elements"], q["setup_query"]["leaf_elements"]
        s2, ql = q["stage_2_query"]["leaf_elements"], q["quotient_query"]["leaf_elements"]
        base = lambda vals: [(int(v) % P, 0) for v in vals]  # noqa: E731
        ext = lambda vals: [(int(vals[i]) % P, int(vals[i + 1]) % P) for i in range(0, len(vals), 2)]  # noqa: E731
        z_off, i_off = 0, 2
        lw_off = i_off + 2 * I
        lm_off = lw_off + 2 * L
        sources = (base(wl[0:V]) + base(wl[V:V + W]) + base(sl[V:V + C]) + base(sl[0:V]) +
                   ext(s2[z_off:i_off]) + ext(s2[i_off:lw_off]) + base(wl[V + W:V + W + M]) +
                   ext(s2[lw_off:lm_off]) + ext(s2[lm_off:]) + base(sl[V + C:V + C + g["lookup_setups"]]) + ext(ql))
        acc = (0, 0)
        off = 0

        def quotening(acc, srcs, vals, at, off):
            den = e_inv(e_sub((xq, 0), at))
            a = (0, 0)
            for f, v, ch in zip(srcs, vals, deep_ch[off:off + len(srcs)]):
                a = e_add(a, e_mul(ch, e_sub(f, tuple(int(t) % P for t in v))))
            return e_add(acc, e_mul(a, den)), off + len(srcs)

        assert len(sources) == len(fx["values_at_z"])
        acc, off = quotening(acc, sources, fx["values_at_z"], z, off)
        z_omega = e_mul_base(z, omega)
        acc, off = quotening(acc, ext(s2[z_off:i_off]), fx["values_at_z_omega"], z_omega, off)
        acc, off = quotening(acc, ext(s2[lw_off:lm_off]) + ext(s2[lm_off:]), fx["values_at_0"], (0, 0), off)
        for at, subset in pi_tuples:
            acc, off = quotening(acc, [(int(wl[col]) % P, 0) for col, _ in subset], [(v, 0) for _, v in subset],
                                 (at, 0), off)
        assert off == len(deep_ch)
        # FRI chain (:2396-2518)
        cur, subidx = acc, idx
        coset_inverse = pow(GEN, P - 2, P)
        x_interp = xq
        expected_len = log_n + (lde_factor.bit_length() - 1) - (cap_size.bit_length() - 1)
        steps = []
        assert len(q["fri_queries"]) == len(schedule)
        for k, (d, fq) in enumerate(zip(schedule, q["fri_queries"])):
            expected_len -= d
            deg = 1 << d
            in_leaf, tree_idx = subidx % deg, subidx >> d
            leaf = [int(v) % P for v in fq["leaf_elements"]]
            steps.append({"expected": (leaf[in_leaf], leaf[deg + in_leaf]), "folded": cur, "leaf": fq["leaf_elements"],
                          "tree_idx": tree_idx, "coset_inverse": coset_inverse, "challenges": fri_ch[k]})
            assert cur == (leaf[in_leaf], leaf[deg + in_leaf]), "FRI element not in the leaf at step %d" % k
            assert len(fq["proof"]) == expected_len
            assert O.verify_proof_over_cap(fq["proof"], caps[k], O.hash_into_leaf(fq["leaf_elements"]), tree_idx), \
                "FRI leaf not in the tree at step %d" % k
            vals = [(leaf[i], leaf[deg + i]) for i in range(deg)]
            base_pow = power_chunks[k]
            ci = coset_inverse
            for ch in fri_ch[k]:
                nxt = []
                for i in range(len(vals) // 2):
                    a, b = vals[2 * i], vals[2 * i + 1]
                    diff = e_mul(e_sub(a, b), ch)
                    diff = e_mul_base(diff, base_pow * interpolation_steps[i] % P * ci % P)
                    nxt.append(e_add(e_add(a, b), diff))
                vals = nxt
                base_pow = base_pow * base_pow % P
                ci = ci * ci % P
            coset_inverse = pow(coset_inverse, 1 << d, P)
            for _ in range(d):
                x_interp = x_interp * x_interp % P
            subidx = tree_idx
            cur = vals[0]
        res = (0, 0)
        for c0, c1 in zip(reversed(mono[0]), reversed(mono[1])):
            res = e_add(e_mul_base(res, x_interp), (int(c0) % P, int(c1) % P))
        assert res == cur, "not equal to the evaluation of final_fri_monomials"
        out_queries.append({"index": idx, "x": xq, "deep": acc, "steps": steps, "final": res})
    return {"beta": beta, "gamma": gamma, "lookup_beta": lookup_beta, "lookup_gamma": lookup_gamma,
            "alpha": alpha, "z": z, "deep_challenge": c, "fri_challenges": fri_ch, "schedule": schedule,
            "num_queries": num_queries, "geometry": g, "queries": out_queries}
