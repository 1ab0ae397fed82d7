"""Flags of the reference (argParser.py:3-73), same names and defaults, plus
the build's own: --data_root (Q8), --device, --mode,
--world_size, --n_max, --train_batch, --train_scenes, --valid_from_seed,
--log_dir, --save_dir, --seed, --use_grid_lstm."""
import argparse


class ArgsParser:
    parser = argparse.ArgumentParser()
    parser.add_argument('--input_size', type=int, default=2)
    parser.add_argument('--rnn_size', type=int, default=128)
    parser.add_argument('--num_layers', type=int, default=2)
    parser.add_argument('--model', type=str, default='lstm')
    parser.add_argument('--batch_size', type=int, default=16)
    parser.add_argument('--seq_length', type=int, default=12)
    parser.add_argument('--pred_len', type=int, default=12)
    parser.add_argument('--obs_len', type=int, default=8)
    parser.add_argument('--num_epochs', type=int, default=10)
    parser.add_argument('--save_every', type=int, default=50)
    parser.add_argument('--grad_clip', type=float, default=10.)
    parser.add_argument('--learning_rate', type=float, default=0.005)
    parser.add_argument('--decay_rate', type=float, default=0.95)
    parser.add_argument('--dropout', type=float, default=0.8)
    parser.add_argument('--embedding_size', type=int, default=64)
    parser.add_argument('--neighborhood_size', type=int, default=64)
    parser.add_argument('--grid_size', type=int, default=4)
    parser.add_argument('--num_freq_blocks', type=int, default=10)
    parser.add_argument('--maxNumPeds', type=int, default=20)
    parser.add_argument('--leaveDataset', type=int, default=2)
    parser.add_argument('--lambda_param', type=float, default=0.0005)
    # build additions
    parser.add_argument('--data_root', type=str, default='data',
                        help='directory holding eth/ and ucy/ (replaces hard-coded paths, Q8)')
    parser.add_argument('--device', type=str, default='cuda')
    parser.add_argument('--mode', choices=('reference', 'train'), default='reference',
                        help="reference: train.py's legs (no loss, as the reference); train: "
                             "RMSProp on the L2 loss over the fold's real scenes, data parallel")
    parser.add_argument('--world_size', type=int, default=0,
                        help='--mode train: expected ranks (torchrun WORLD_SIZE; 0: any)')
    parser.add_argument('--n_max', type=int, default=0,
                        help='--mode train: pedestrian padding Nmax (0: the largest scene, '
                             'rounded up to 16; larger scenes are left out)')
    parser.add_argument('--train_batch', type=int, default=256,
                        help='--mode train: scenes per global step (a multiple of the ranks)')
    parser.add_argument('--loss', choices=('l2', 'nll'), default='l2',
                        help='--mode train: 1/2 squared error of the predictions, or the '
                             'bivariate-Gaussian NLL with a learned per-step head')
    parser.add_argument('--train_scenes', type=int, default=0,
                        help='--mode train: distinct scenes used (0: all of the fold)')
    parser.add_argument('--valid_from_seed', type=int, default=0,
                        help="validation leg from the file's first frame (the reference starts "
                             "at frame 0, which the ETH/UCY frame keys never hit)")
    parser.add_argument('--use_grid_lstm', type=int, default=0,
                        help="run the vis/loc encoder's GridLSTMCell in every frame and feed its "
                             "output as st_embeddings (train.py:201-207; 0: the reference, whose "
                             "encoder outputs are overridden by feeds, quirk Q5)")
    parser.add_argument('--log_dir', type=str, default='log')
    parser.add_argument('--seed', type=int, default=0)
    parser.add_argument('--save_dir', type=str, default='',
                        help='write TF-bundle checkpoints every --save_every batches (train.py:330-343)')
