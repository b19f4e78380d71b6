timeout -k 10 1000 python -u tools/race_full.py > gpurun_out/r3race.txt 2>&1
