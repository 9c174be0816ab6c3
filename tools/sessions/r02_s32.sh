set -u
bash tools/sweep_resumable.sh 14 100 r02_sweep_medium_s16o14_v11 && bash tools/sweep_resumable.sh 1 250 r02_sweep_medium_s16o1_v12 && bash tools/sweep_resumable.sh 3 250 r02_sweep_medium_s16o3_v12
