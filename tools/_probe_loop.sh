set -o pipefail
timeout -k 10 300 python -u tools/_probe_loop.py
