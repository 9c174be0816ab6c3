set -u
bash tools/sweep_resumable.sh 10 150 r02_sweep_medium_s16o10_v11 && bash tools/sweep_resumable.sh 14 300 r02_sweep_medium_s16o14_v11 && bash tools/sweep_resumable.sh 1 500 r02_sweep_medium_s16o1_v12
