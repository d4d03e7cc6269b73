"""CPU: the message-passing layer's untracked LDS-DMA (gemm_x6.hpp ``glds16_untracked``: inline-asm
``global_load_lds_dwordx4`` the compiler does not see) is ordered only by the kernel's own explicit
``s_waitcnt vmcnt`` before the barrier that publishes the stage.  That protocol is sound only if no
compiler-issued vector-memory instruction is in flight between a DMA and the wait that covers it: an
extra load or store there would change what the hand-written count means (and a store may complete out of
order with the DMA).  This test disassembles every ``mp_layer_kernel`` instantiation (and the pair-operand
``wo_readout_kernel``) in the built
libwdmpnn.so (gfx950 code object) and walks the control-flow graph from each DMA: every path must reach an
``s_waitcnt`` with a vmcnt field before it meets any other vector-memory instruction."""
import os
import re
import shutil
import subprocess

import pytest

LLVM = '/opt/rocm/lib/llvm/bin'
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'polymer-chemprop_amd',
                   'chemprop_amd', 'libwdmpnn.so')
VMEM = re.compile(r'^(global_|buffer_|flat_|scratch_)')
INSN = re.compile(r'^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):')
TARGET = re.compile(r'<[^>]*\+0x([0-9a-f]+)>')


def _tools():
    need = [os.path.join(LLVM, t) for t in ('llvm-objcopy', 'clang-offload-bundler', 'llvm-objdump')]
    return need if all(os.path.exists(t) for t in need) and os.path.exists(LIB) else None


@pytest.fixture(scope='module')
def layer_kernels(tmp_path_factory):
    tools = _tools()
    if tools is None:
        pytest.skip('ROCm LLVM tools or the built libwdmpnn.so not present')
    objcopy, bundler, objdump = tools
    d = tmp_path_factory.mktemp('co')
    fat, co = str(d / 'fat.bin'), str(d / 'co.o')
    subprocess.run([objcopy, f'--dump-section=.hip_fatbin={fat}', LIB, str(d / 'host.o')], check=True)
    subprocess.run([bundler, '--type=o', f'--input={fat}', '--targets=hipv4-amdgcn-amd-amdhsa--gfx950',
                    f'--output={co}', '--unbundle'], check=True)
    table = subprocess.run([objdump, '-t', co], check=True, capture_output=True, text=True).stdout
    # (and the W_o kernel's pair instantiations, PAIRS = true: the same untracked copies, gemm_x6.hpp
    # h2_mainloop_pairs)
    syms = sorted({ln.split()[-1] for ln in table.split('\n') if ' F ' in ln and not ln.split()[-1].endswith('.kd')
                   and ('mp_layer_kernel' in ln or ('wo_readout_kernel' in ln and 'Lb1EEEv' in ln))})
    assert syms, 'no mp_layer_kernel in the code object'
    text = subprocess.run([objdump, '-d', '--mcpu=gfx950', '--disassemble-symbols=' + ','.join(syms), co],
                          check=True, capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for ln in text.split('\n'):
        m = re.match(r'^([0-9a-f]+) <(\S+)>:', ln)
        if m:
            cur = funcs.setdefault(m.group(2), {'base': int(m.group(1), 16), 'insns': []})
            continue
        m = INSN.match(ln)
        if cur is not None and m:
            t = TARGET.search(ln)
            cur['insns'].append((int(m.group(3), 16), m.group(1), m.group(2),
                                 cur['base'] + int(t.group(1), 16) if t else None))
    shutil.rmtree(str(d), ignore_errors=True)
    return funcs


def _walk(insns, start):
    """Every path from the DMA at insns[start]: the vector-memory instructions met before a vmcnt wait, and
    the waits that end the paths."""
    index = {a: i for i, (a, *_) in enumerate(insns)}
    bad, waits, seen, todo = [], set(), set(), [start + 1]
    while todo:
        i = todo.pop()
        while i < len(insns) and i not in seen:
            seen.add(i)
            addr, mnem, ops, tgt = insns[i]
            if mnem == 's_waitcnt' and 'vmcnt' in ops:
                waits.add(ops)
                break
            if VMEM.match(mnem) and mnem != 'global_load_lds_dwordx4':
                bad.append((hex(addr), mnem, ops))
            if mnem == 's_endpgm':
                break
            if mnem == 's_branch':
                i = index[tgt]
                continue
            if mnem.startswith('s_cbranch') and tgt is not None:
                todo.append(index[tgt])
            i += 1
    return bad, waits


def test_layer_kernels_have_no_vector_memory_between_dma_and_its_wait(layer_kernels):
    checked = 0
    for name, f in layer_kernels.items():
        insns = f['insns']
        dmas = [i for i, x in enumerate(insns) if x[1] == 'global_load_lds_dwordx4']
        assert dmas, f'{name}: no LDS-DMA (the mainloop changed: update this test)'
        for i in dmas:
            bad, waits = _walk(insns, i)
            assert not bad, (name, hex(insns[i][0]), bad[:4])
            assert waits, (name, hex(insns[i][0]), 'a DMA reaches the end without a vmcnt wait')
            checked += 1
    assert checked >= 8 * len(layer_kernels) // 2


def test_walker_finds_a_load_on_a_branch_path():
    """The checker itself: a load reached through a taken branch (the loop back-edge shape) is reported,
    a path that meets the wait first is not."""
    insns = [(0, 'global_load_lds_dwordx4', 'v[0:1], off', None),
             (4, 's_cbranch_scc1', '2', 16),
             (8, 's_waitcnt', 'vmcnt(0)', None),
             (12, 's_endpgm', '', None),
             (16, 'buffer_load_dwordx4', 'v[2:5], v0, s[0:3], 0 offen', None),
             (20, 's_branch', '65531', 8)]
    bad, waits = _walk(insns, 0)
    assert bad == [('0x10', 'buffer_load_dwordx4', 'v[2:5], v0, s[0:3], 0 offen')] and waits == {'vmcnt(0)'}
    bad, _ = _walk([insns[0], insns[2], insns[4], insns[3]], 0)  # the load after the wait
    assert not bad
