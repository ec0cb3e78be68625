import sys; sys.path.insert(0,'tests'); sys.path.insert(0,'.')
from hocuspocus_amd import Engine
import oracle
u=bytes.fromhex('02038080010000020a038480800104010001858080800800000200'); sv=bytes.fromhex('028080010a858080800801')
for compat in (False, True):
    e=Engine(0, compat135=compat)
    print('diff', compat, e.diff_update_batch([u],[sv]), oracle.diff_update(u, sv))
    print('sv', e.encode_state_vector_from_update_batch([u]), oracle.encode_state_vector_from_update(u))
    e.close()
from tools import synth
a,o,s,so=synth.text_states(4, seed=3)
docs=synth.split(a,o); svs=synth.split(s,so)
e=Engine(0)
print(e.encode_state_vector_from_update_batch(docs)[:2])
print(e.diff_update_batch(docs, svs)[0][0])
print(docs[0][:60].hex())
