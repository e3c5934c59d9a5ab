"""gfx950 Equihash(200,9) solver vs the CPU golden solver/verifier."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver(gpu):
    """The private-slot solver (equihash_ps.hip)."""
    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    s = EquihashSolver(num_inst=4, device=0)
    yield s
    del s
    torch.cuda.empty_cache()


def test_blake2b_h0_matches_cpu(core):
    from nodexa_chain_core_amd.ops.equihash import blake2b_h0

    # h0 derived from the parameter block must reproduce the CPU BLAKE2b digest
    p = core.EquihashParams(200, 9)
    assert len(blake2b_h0()) == 8
    assert core.blake2b(b"x", 50, p.personal) != core.blake2b(b"x", 50, None)


def test_gpu_solutions_valid_and_match_cpu(core, solver):
    inputs = [bytes(80) + i.to_bytes(32, "little") for i in range(4)]
    gpu = solver.solve(inputs)  # every solution already CPU-verified inside collect()
    st = solver.stats()
    assert st["stage_dropped"] == 0 and st["largest_bucket"] <= st["cap"], st  # no staged bucket over its cap
    assert sum(st["dropped_per_level"]) < 64, st  # segment / staging overflow stays rare
    assert min(st["rows_per_level"]) > 1_900_000, st
    total_gpu = sum(len(s) for s in gpu)
    total_cpu = 0
    for inp, g in zip(inputs, gpu):
        cpu, _ = core.equihash_solve_cpu(core.EquihashParams(200, 9), inp, 16, 0)
        total_cpu += len(cpu)
        for s in g:
            assert s in cpu  # same canonical form as the golden solver
    assert total_cpu > 0
    assert total_gpu >= total_cpu - 1  # bucket-capacity drops may lose at most a rare solution


def test_solver_exactly_matches_cpu_on_16_inputs(core, gpu):
    """The solver is lossless: every device-side cap (segment, staging, chain, candidate) is
    counted per instance and a counted instance is re-solved on the golden solver, so the solution
    sets equal the CPU solver's on every input — and no instance needed that here."""
    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    s = EquihashSolver(num_inst=8, device=0)
    p = core.EquihashParams(200, 9)
    inputs = [bytes([0x5A]) * 80 + i.to_bytes(32, "little") for i in range(16)]
    gpu = s.solve(inputs[:8]) + s.solve(inputs[8:])
    total = 0
    for inp, g in zip(inputs, gpu):
        cpu, _ = core.equihash_solve_cpu(p, inp, 16, 0)
        assert sorted(map(tuple, g)) == sorted(map(tuple, cpu)), inp[-32:].hex()
        total += len(g)
    assert total > 8
    assert s.fallbacks == 0, str(s.fallback_log)
    del s
    torch.cuda.empty_cache()


def test_gpu_batch_verify_matches_cpu(core, solver):
    from nodexa_chain_core_amd.ops.equihash import verify_solutions

    p = core.EquihashParams(200, 9)
    inputs = [bytes([3]) * 80 + i.to_bytes(32, "little") for i in range(4)]
    sols = solver.solve(inputs)
    batch_in, batch_sol, expect = [], [], []
    for inp, ss in zip(inputs, sols):
        for s in ss:
            packed = core.equihash_pack(p, s)
            batch_in.append(inp)
            batch_sol.append(packed)
            expect.append(True)
            # corruptions the CPU verifier rejects: a flipped leaf index, swapped subtrees, a repeat
            for mut in (lambda x: x[:1] + [x[1] ^ 1] + x[2:], lambda x: x[256:] + x[:256], lambda x: x[:511] + x[:1]):
                bad = mut(list(s))
                batch_in.append(inp)
                batch_sol.append(core.equihash_pack(p, bad))
                expect.append(bool(core.equihash_verify(p, inp, bad)[0]))
    assert any(expect) and not all(expect)
    assert verify_solutions(batch_in, batch_sol, device=0) == expect


def test_gpu_repeatable(solver):
    inputs = [bytes([7]) * 112 for _ in range(4)]
    a = solver.solve(inputs)
    b = solver.solve(inputs)
    canon = [sorted(map(tuple, x)) for x in a]
    assert canon == [sorted(map(tuple, x)) for x in b]
    # identical inputs in one batch: the same solution set (the order in which the
    # reconstruct workgroups append them is not fixed)
    assert all(x == canon[0] for x in canon)
