"""XBot-L humanoid configuration — the 12-DOF profile of SURVEY.md Appendix A.

Same class/field names as the reference ``XBotLCfg`` / ``XBotLCfgPPO``
(humanoid/envs/custom/humanoid_config.py:33-505) so user code that reads or overrides fields keeps
working.  Differences, all forced by the fork's internal inconsistency:
  * the fork describes an 18-DOF "D11_X" robot whose URDF is not shipped; this profile is the
    shipped 12-DOF XBot-L (num_actions 12, obs frame 47, privileged frame 73);
  * PD gains come from the XBot-L block commented in humanoid/scripts/sim2sim.py:306-309
    (the fork's stiffness keys do not match XBot-L joint names and would give zero gains);
  * default joint angles are all 0 and the spawn height 0.95 m (BUILD-DEFINED);
  * new `sim.hg` section: parameters of this build's contact solver (PhysX TGS has no
    equivalent knobs) and the model armature.
Everything else keeps the reference value.
"""
from humanoid.envs.base.base_config import BaseConfig


class XBotLCfg(BaseConfig):
    class env:
        frame_stack = 15                  # :43
        c_frame_stack = 3                 # :45
        num_actions = 12
        num_single_obs = 47
        num_observations = int(frame_stack * num_single_obs)       # 705
        single_num_privileged_obs = 73
        num_privileged_obs = int(c_frame_stack * single_num_privileged_obs)   # 219
        env_spacing = 3.0
        send_timeouts = True
        num_envs = 4096
        episode_length_s = 24
        use_ref_actions = False
        num_observation_history_len = 1
        # data parallel (new): this shard holds global envs [env_offset, env_offset +
        # num_envs) of num_envs_total (None: num_envs).  Philox draws, plane-grid origins, terrain
        # levels / types and the creation-time DR are functions of the global env id, so a sharded
        # run is the single run on num_envs_total envs, split.
        env_offset = 0
        num_envs_total = None

    class safety:
        pos_limit = 1.0
        vel_limit = 1.0
        torque_limit = 0.85

    class asset:
        file = "{LEGGED_GYM_ROOT_DIR}/model/xbotl_model.json"   # compiled from XBot-L.urdf
        name = "XBot-L"
        foot_name = "ankle_roll"
        knee_name = "knee"
        disable_gravity = False
        collapse_fixed_joints = True
        default_dof_drive_mode = 3
        terminate_after_contacts_on = ["base_link"]
        penalize_contacts_on = ["base_link"]
        self_collisions = 0
        flip_visual_attachments = False
        replace_cylinder_with_capsule = False
        fix_base_link = False
        density = 0.001
        angular_damping = 0.0
        linear_damping = 0.0
        max_angular_velocity = 1000.0
        max_linear_velocity = 1000.0
        armature = 0.0
        thickness = 0.01

    class terrain:
        mesh_type = "plane"               # 'plane' | 'heightfield' | 'trimesh'
        seed = None                       # heightfield generator seed (None: the run seed)
        horizontal_scale = 0.1
        vertical_scale = 0.005
        border_size = 25
        curriculum = False
        measure_heights = False
        measured_points_x = [-0.8, -0.7, -0.6, -0.5, -0.4, -0.3, -0.2, -0.1, 0.0, 0.1, 0.2, 0.3, 0.4,
                             0.5, 0.6, 0.7, 0.8]
        measured_points_y = [-0.5, -0.4, -0.3, -0.2, -0.1, 0.0, 0.1, 0.2, 0.3, 0.4, 0.5]
        selected = False
        terrain_kwargs = None
        static_friction = 0.6
        dynamic_friction = 0.6
        terrain_length = 8.0
        terrain_width = 8.0
        num_rows = 20
        num_cols = 20
        max_init_terrain_level = 10
        terrain_proportions = [0.2, 0.2, 0.4, 0.1, 0.1, 0, 0]
        restitution = 0.0
        slope_treshold = 0.75

    class noise:
        add_noise = True
        noise_level = 0.6

        class noise_scales:
            dof_pos = 0.05
            dof_vel = 0.5
            ang_vel = 0.1
            lin_vel = 0.05
            quat = 0.03
            height_measurements = 0.1
            gravity = 0.05

    class viewer:
        ref_env = 0
        pos = [10, 0, 6]
        lookat = [11.0, 5, 3.0]

    class init_state:
        pos = [0.0, 0.0, 0.95]
        rot = [0.0, 0.0, 0.0, 1.0]
        lin_vel = [0.0, 0.0, 0.0]
        ang_vel = [0.0, 0.0, 0.0]
        default_joint_angles = {
            "left_leg_roll_joint": 0.0, "left_leg_yaw_joint": 0.0, "left_leg_pitch_joint": 0.0,
            "left_knee_joint": 0.0, "left_ankle_pitch_joint": 0.0, "left_ankle_roll_joint": 0.0,
            "right_leg_roll_joint": 0.0, "right_leg_yaw_joint": 0.0, "right_leg_pitch_joint": 0.0,
            "right_knee_joint": 0.0, "right_ankle_pitch_joint": 0.0, "right_ankle_roll_joint": 0.0,
        }

    class control:
        # substring match on joint names, as _init_buffers does (humanoid_env.py:285-297)
        stiffness = {"leg_roll": 200.0, "leg_pitch": 350.0, "leg_yaw": 200.0, "knee": 350.0, "ankle": 15.0}
        damping = {"leg_roll": 10, "leg_pitch": 10, "leg_yaw": 10, "knee": 10, "ankle": 10}
        action_scale = 0.25
        decimation = 10

    class sim:
        dt = 0.001
        substeps = 1
        gravity = [0.0, 0.0, -9.81]
        up_axis = 1

        class physx:
            num_threads = 10
            solver_type = 1
            num_position_iterations = 4
            num_velocity_iterations = 1
            contact_offset = 0.01
            rest_offset = 0.0
            bounce_threshold_velocity = 0.1
            max_depenetration_velocity = 1.0
            max_gpu_contact_pairs = 2 ** 23
            default_buffer_size_multiplier = 5
            contact_collection = 2

        class hg:
            # projected Gauss-Seidel sweeps per substep; None = the reference's solver budget,
            # physx.num_position_iterations + physx.num_velocity_iterations (4 + 1)
            pgs_iterations = None
            baumgarte = 0.2            # fraction of penetration corrected per substep
            # joint-space armature: the asset's 0 (asset.armature, humanoid_config.py:118 of the
            # reference); the PD damping term is integrated implicitly, which keeps kd = 10 on
            # the light foot stable at dt = 1 ms (0.01 = the MJCF's value, XBot-L.xml:37-39)
            armature = 0.0
            joint_friction = True      # URDF joint friction: 0.1 N m on the ankles (XBot-L.urdf:1675-1677)

    class domain_rand:
        randomize_friction = True
        friction_range = [0.1, 2.0]
        randomize_base_mass = True
        added_mass_range = [-5.0, 5.0]
        push_robots = True
        push_interval_s = 4
        max_push_vel_xy = 0.2
        max_push_ang_vel = 0.4
        # push-recovery curriculum (BUILD-DEFINED, config 5; the reference only has fixed pushes,
        # humanoid_env.py:665-681): push magnitudes ramp linearly with the PPO iteration
        push_curriculum = False
        push_curriculum_iterations = 1000
        max_push_vel_xy_final = 1.0
        max_push_ang_vel_final = 1.0
        dynamic_randomization = 0.02

    class commands:
        curriculum = False
        max_curriculum = 1.0
        num_commands = 4
        resampling_time = 8.0
        heading_command = True

        class ranges:
            lin_vel_x = [-0.3, 0.6]
            lin_vel_y = [-0.3, 0.3]
            ang_vel_yaw = [-0.3, 0.3]
            heading = [-3.14, 3.14]

    class rewards:
        base_height_target = 0.94
        min_dist = 0.2
        max_dist = 0.5
        target_joint_pos_scale = 0.17
        target_feet_height = 0.1
        cycle_time = 0.64
        only_positive_rewards = True
        tracking_sigma = 5
        max_contact_force = 700

        class scales:
            joint_pos = 1.6
            feet_clearance = 1.0
            feet_contact_number = 1.2
            feet_air_time = 1.0
            foot_slip = -0.05
            feet_distance = 0.2
            knee_distance = 0.2
            feet_contact_forces = -0.01
            tracking_lin_vel = 1.2
            tracking_ang_vel = 1.1
            vel_mismatch_exp = 0.5
            low_speed = 0.2
            track_vel_hard = 0.5
            default_joint_pos = 0.5
            orientation = 1.0
            base_height = 0.2
            base_acc = 0.2
            action_smoothness = -0.002
            torques = -1e-5
            dof_vel = -5e-4
            dof_acc = -1e-7
            collision = -1.0
            termination = -0.0
            feet_stumble = -0.0
            action_rate = -0.0
            stand_still = -0.0

    class normalization:
        class obs_scales:
            lin_vel = 2.0
            ang_vel = 1.0
            dof_pos = 1.0
            dof_vel = 0.05
            quat = 1.0
            height_measurements = 5.0

        clip_observations = 18.0
        clip_actions = 18.0


class XBotLCfgPPO(BaseConfig):
    seed = 5
    runner_class_name = "OnPolicyRunner"

    class policy:
        init_noise_std = 1.0
        actor_hidden_dims = [512, 256, 128]
        critic_hidden_dims = [768, 256, 128]
        policy_dtype = "fp32"      # "bf16": bf16 activations + matrix-core GEMMs, fp32 master weights (config 5)

    class algorithm:
        value_loss_coef = 1.0
        use_clipped_value_loss = True
        clip_param = 0.2
        entropy_coef = 0.001
        learning_rate = 1e-5
        schedule = "adaptive"
        num_learning_epochs = 2
        gamma = 0.994
        lam = 0.9
        num_mini_batches = 4
        desired_kl = 0.01
        max_grad_norm = 1.0

    class runner:
        policy_class_name = "ActorCritic"
        algorithm_class_name = "PPO"
        num_steps_per_env = 60
        storage_obs_dtype = "fp32"  # "fp16": observation buffers of the rollout storage (config 5)
        max_iterations = 3001
        save_interval = 100
        experiment_name = "XBot_ppo"
        run_name = ""
        resume = False
        load_run = -1
        checkpoint = -1
        resume_path = None
