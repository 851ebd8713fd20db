"""Command line of the reference (main.py:17-109) on the GPU env.

    python -m vmp.main -a ppo -c config/10.yml -r wr -e -w weights-10/ppo-wr.pt -o out.json

Same flags, same YAML schema (`environment:` section -> Config, `agents:
<name>:` -> the agent's config), same seeding (main.py:40-45), same
load-or-learn-then-save weights logic (main.py:65-77) and `agent.test` eval
(main.py:79-82); `run(Args)` returns the Record as the reference's does (the
exp_* drivers call it). Additions: `--envs N` trains PPO on N batched GPU envs
(the reference trains one), `--device`. The drlvmp / convex / rainbow agents
are out of scope and raise.
"""
import argparse
import os
import random
from dataclasses import dataclass, fields

import numpy as np
import torch

from .agents import BestFitAgent, FirstFitAgent
from .config import Config


@dataclass
class Args:
    agent: str
    reward: str
    config: dict
    logdir: str = None
    output: str = None
    silent: bool = False
    jobname: str = None
    weightspath: str = None
    eval: bool = False
    debug: bool = False
    envs: int = 1
    device: str = "cuda"


def _known(cls, d):
    names = {f.name for f in fields(cls)}
    return {k: v for k, v in (d or {}).items() if k in names}


def make_agent(name, env, agent_config):
    if name == "ppo":
        from .ppo import PPOAgent, PPOConfig
        return PPOAgent(env, PPOConfig(**_known(PPOConfig, agent_config)))
    if name == "firstfit":
        return FirstFitAgent(env)
    if name == "bestfit":
        return BestFitAgent(env)
    raise ValueError(f"Agent cannot be {name}: only ppo, firstfit and bestfit run on this "
                     "build (drlvmp / convex / rainbow are out of scope)")


def run(args: Args):
    """main.py:34-86."""
    from .env import VmEnv
    config = args.config
    env_config = dict(config["environment"])
    env_config["reward_function"] = args.reward
    agent_config = config.get("agents", {}).get(args.agent, {}) or {}

    seed = env_config["seed"]
    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)

    env = VmEnv(Config(**_known(Config, env_config)), device=args.device)
    agent = make_agent(args.agent, env, agent_config)
    if args.logdir and args.jobname:
        agent.set_log(jobname=args.jobname, logdir=args.logdir)

    def learn():
        if args.agent == "ppo" and args.envs > 1:
            # batched training on N GPU envs, then the weights go to the N=1 agent
            from .batched import BatchedVmEnv
            benv = BatchedVmEnv(env.config, args.envs, device=env._b.device)
            trainer = make_agent("ppo", benv, agent_config)
            trainer.learn()
            agent.model.load_state_dict(trainer.model.state_dict())
            benv.close()
        else:
            agent.learn()

    if args.weightspath:
        print(f"Weights: {args.weightspath}...")
        if os.path.exists(args.weightspath):
            agent.load_model(args.weightspath)
        else:
            learn()
    else:
        learn()
    if args.weightspath and not os.path.exists(args.weightspath):
        agent.save_model(args.weightspath)
        print(f"Weights saved to {args.weightspath}.")
    record = None
    if args.eval:
        record = agent.test(show=not args.silent, output=args.output, debug=args.debug)
    agent.end_log()
    env.close()
    return record


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-a", "--agent", required=True,
                   choices=["ppo", "firstfit", "bestfit", "convex", "rainbow", "drlvmp"],
                   help="Choose an agent to train or evaluate.")
    p.add_argument("-c", "--config", default="config/10.yml",
                   help="Configuration for environment and agent")
    p.add_argument("-r", "--reward", default="wr", choices=["wr", "ut", "kl"],
                   help="wr: waiting ratio, ut: utilization, kl: kl divergence")
    p.add_argument("-d", "--debug", action="store_true", help="Print step-by-step debug info")
    p.add_argument("-l", "--logdir", help="Directory of tensorboard logs")
    p.add_argument("-j", "--jobname", help="Job name in tensorboard")
    p.add_argument("-o", "--output", default="./output.json", help="Path of result json file")
    p.add_argument("-w", "--weightspath", help="path of ppo's weights to load or to save")
    p.add_argument("-e", "--eval", action="store_true",
                   help="to evaluate a model instead of training")
    p.add_argument("-s", "--silent", default=False, action="store_true",
                   help="Do not print summary of the model")
    p.add_argument("--envs", type=int, default=1, help="batched GPU envs for PPO training")
    p.add_argument("--device", default="cuda")
    a = p.parse_args(argv)
    import yaml
    with open(a.config) as f:
        cfg = yaml.safe_load(f)
    return Args(agent=a.agent, reward=a.reward, config=cfg, logdir=a.logdir, output=a.output,
                silent=a.silent, jobname=a.jobname, weightspath=a.weightspath, eval=a.eval,
                debug=a.debug, envs=a.envs, device=a.device)


if __name__ == "__main__":
    run(parse())
