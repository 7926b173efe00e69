from dbindex_amd import fasta
from dbindex_amd.engine import Engine
from dbindex_amd.params import DBIndexSearchParams
import sys
pp = fasta.config(sys.argv[1] if len(sys.argv) > 1 else "human", with_defs=False)
cp = DBIndexSearchParams.trypsin(2).to_c()
with Engine(cp) as eng:
    for k in range(7):
        st = eng.build(pp)
        print(k, sorted({n for n, _, _ in eng.stage_times()}), st.n_kept, flush=True)
