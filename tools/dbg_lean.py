"""Ad-hoc GPU check: a few merge inputs through the engine vs the oracle (hex dump)."""
import sys; sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from hocuspocus_amd import Engine
import oracle
cases = [['000102010001', '000109010001'],
         ['0001c8010219041604', '0000', '0000', '0002020216000b0401011601'],
         ['0000', '0003020404030d030f021d05c801020b01090402011804', '000101010602'],
         ['000102010001', '000102010101'],
         ['01010500040101740568656c6c6f00', '000105010001'],
         ['01010500040101740568656c6c6f00', '01010505840500016100', '000105010001']]
e = Engine(0)
for c in cases:
    us = [bytes.fromhex(x) for x in c]
    l0 = e.stats().docs_lean
    g = e.merge_updates_batch([us])[0]
    o = oracle.merge_updates(us)
    print('OK ' if g == o else 'BAD', e.stats().docs_lean - l0, g[0], g[1].hex(), '| oracle', o[0], o[1].hex())
