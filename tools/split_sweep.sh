bash tools/ab.sh 2
bash tools/ab.sh 1 --kind mixed --steps 2
