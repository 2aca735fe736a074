# round-4 evidence call 2 (r04t): PMC passes of C2 / C4 / C5, the C4 and C5 lines
T=r04t
TAG=$T bash scripts/gpu.sh pmc:c2 pmc:c4 pmc:c5 bench:c4 bench:c5
