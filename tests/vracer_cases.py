"""The reference's examples/learning/reinforcement/cartpole/run-vracer.py
configuration, on the device CartPole environment kernel."""
import korali


def cartpole_vracer(max_generations=50, environments=1, hidden=32, policy="Clipped Normal", kernel="CartPole"):
    """run-vracer.py with its defaults (50 generations, 1 concurrent
    environment, two 32-wide tanh layers, Clipped Normal policy); the host
    `env` function replaced by the device CartPole kernel."""
    e = korali.Experiment()
    e["Problem"]["Type"] = "Reinforcement Learning / Continuous"
    if kernel is None:
        e["Problem"]["Environment Function"] = lambda s: None  # a host environment
    else:
        e["Problem"]["Environment Kernel"] = kernel
    e["Problem"]["Environment Count"] = 3
    e["Problem"]["Actions Between Policy Updates"] = 1
    for i, n in enumerate(["Cart Position", "Cart Velocity", "Pole Angle", "Pole Angular Velocity"]):
        e["Variables"][i]["Name"] = n
        e["Variables"][i]["Type"] = "State"
    e["Variables"][4]["Name"] = "Force"
    e["Variables"][4]["Type"] = "Action"
    e["Variables"][4]["Lower Bound"] = -10.0
    e["Variables"][4]["Upper Bound"] = +10.0
    e["Variables"][4]["Initial Exploration Noise"] = 1.0
    e["Solver"]["Type"] = "Agent / Continuous / VRACER"
    e["Solver"]["Mode"] = "Training"
    e["Solver"]["Experiences Between Policy Updates"] = 1
    e["Solver"]["Episodes Per Generation"] = 10
    e["Solver"]["Concurrent Environments"] = environments
    e["Solver"]["Experience Replay"]["Start Size"] = 1000
    e["Solver"]["Experience Replay"]["Maximum Size"] = 10000
    e["Solver"]["Discount Factor"] = 0.99
    e["Solver"]["Learning Rate"] = 1e-4
    e["Solver"]["Mini Batch"]["Size"] = 32
    e["Solver"]["State Rescaling"]["Enabled"] = False
    e["Solver"]["Reward"]["Rescaling"]["Enabled"] = False
    e["Solver"]["Neural Network"]["Engine"] = "OneDNN"
    e["Solver"]["Neural Network"]["Optimizer"] = "Adam"
    e["Solver"]["Policy"]["Distribution"] = policy
    e["Solver"]["Neural Network"]["Hidden Layers"][0]["Type"] = "Layer/Linear"
    e["Solver"]["Neural Network"]["Hidden Layers"][0]["Output Channels"] = hidden
    e["Solver"]["Neural Network"]["Hidden Layers"][1]["Type"] = "Layer/Activation"
    e["Solver"]["Neural Network"]["Hidden Layers"][1]["Function"] = "Elementwise/Tanh"
    e["Solver"]["Neural Network"]["Hidden Layers"][2]["Type"] = "Layer/Linear"
    e["Solver"]["Neural Network"]["Hidden Layers"][2]["Output Channels"] = hidden
    e["Solver"]["Neural Network"]["Hidden Layers"][3]["Type"] = "Layer/Activation"
    e["Solver"]["Neural Network"]["Hidden Layers"][3]["Function"] = "Elementwise/Tanh"
    e["Solver"]["Termination Criteria"]["Max Generations"] = max_generations
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    e["Random Seed"] = 1337
    return e
