set -u
bash tools/sweep_resumable.sh 14 120 r02_sweep_medium_s16o14_v11 && bash tools/sweep_resumable.sh 1 420 r02_sweep_medium_s16o1_v12 && bash tools/sweep_resumable.sh 3 400 r02_sweep_medium_s16o3_v12
