# final HEAD check: full GPU suite + smoke, then the 4-vs-8 chain A/B
set -u
bash tools/_g34.sh || exit 1
bash tools/_g40.sh
