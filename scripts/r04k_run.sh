# round-4 GPU call (r04p): A/B of the tree-sum LayerNorm in the clip-group loop (C2)
T=r04p
TAG=$T ROUNDS=3 bash scripts/ab.sh c2 ab/libggd_mx.so ab/libggd_lntree.so
