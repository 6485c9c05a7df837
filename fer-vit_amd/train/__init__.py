"""Training steps of the reference trainers (`train/train_*.py` train_epoch / evaluate /
get_optimizer_groups) on the MI355X modules, plus the data-parallel launcher
(`train.ddp`). Same function names and arguments as the reference modules; no per-step host
synchronisation (metrics cross to the host once per epoch)."""
