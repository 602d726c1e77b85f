variable "hostname" {
  description = "Host name given to the node."
  type        = string

  validation {
    condition     = length(regexall("^[A-Za-z0-9]([-A-Za-z0-9.]{0,251}[A-Za-z0-9])?$", var.hostname)) > 0
    error_message = "hostname must be a DNS host name."
  }
}

variable "rancher_api_url" {
  description = "Base URL of the Rancher server (the cluster manager's rancher_url output)."
  type        = string

  validation {
    condition     = length(regexall("^https?://[][A-Za-z0-9._:-]+(/[A-Za-z0-9._/-]*)?$", var.rancher_api_url)) > 0
    error_message = "rancher_api_url must be an http(s) URL."
  }
}

variable "k8s_distribution" {
  description = "the cluster's distribution: rke2 joins with the server's system-agent installer, rke1 with docker run rancher/rancher-agent"
  type        = string
  default     = "rke2"

  validation {
    condition     = contains(["rke2", "rke1"], var.k8s_distribution)
    error_message = "k8s_distribution must be rke2 or rke1."
  }
}

variable "rancher_cluster_registration_token" {
  description = "Registration token of the cluster the node joins."
  type        = string
  sensitive   = true

  validation {
    condition     = length(regexall("^[A-Za-z0-9._:-]{1,512}$", var.rancher_cluster_registration_token)) > 0
    error_message = "rancher_cluster_registration_token must be a Rancher registration token."
  }
}

variable "rancher_cluster_ca_checksum" {
  description = "SHA-256 of the Rancher CA bundle, pinned by the agent."
  type        = string

  validation {
    condition     = length(regexall("^[A-Za-z0-9]{0,128}$", var.rancher_cluster_ca_checksum)) > 0
    error_message = "rancher_cluster_ca_checksum must be a hex checksum (or empty)."
  }
}

variable "rancher_host_labels" {
  description = "A single-key map: {worker|etcd|control = \"true\"}"
  type        = map(string)

  validation {
    condition     = length(var.rancher_host_labels) == 1 && contains(["worker", "etcd", "control"], keys(var.rancher_host_labels)[0])
    error_message = "rancher_host_labels must hold exactly one of worker, etcd or control."
  }
}

variable "docker_engine_install_url" {
  description = "The URL to the shell script to install the docker engine."
  type        = string
  default     = "https://releases.rancher.com/install-docker/24.0.sh"

  validation {
    condition     = length(regexall("^(https?://[][A-Za-z0-9._:-]+(/[A-Za-z0-9._/~%+=-]*)?)?$", var.docker_engine_install_url)) > 0
    error_message = "docker_engine_install_url must be an http(s) URL (or empty)."
  }
}

variable "docker_install_sha256" {
  description = "SHA-256 the downloaded runtime install script must match (empty: not checked)."
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("^[A-Fa-f0-9]{0,64}$", var.docker_install_sha256)) > 0
    error_message = "docker_install_sha256 must be a sha256 hex digest (or empty)."
  }
}

variable "rancher_agent_image" {
  description = "The Rancher Agent image to use."
  type        = string
  default     = "rancher/rancher-agent:v2.10.3"

  validation {
    condition     = length(regexall("^[A-Za-z0-9][A-Za-z0-9._/:@-]{0,254}$", var.rancher_agent_image)) > 0
    error_message = "rancher_agent_image must be a container image reference."
  }
}

variable "rancher_registry" {
  description = "The docker registry to use for rancher server and agent images"
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("^([A-Za-z0-9][A-Za-z0-9._/:@-]{0,254})?$", var.rancher_registry)) > 0
    error_message = "rancher_registry must be a registry host (or empty)."
  }
}

variable "rancher_registry_username" {
  description = "The username to login as."
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("['\"\\\\]", var.rancher_registry_username)) == 0
    error_message = "rancher_registry_username must not contain quotes or backslashes."
  }
}

variable "rancher_registry_password" {
  description = "The password to use."
  type        = string
  default     = ""
  sensitive   = true

  validation {
    condition     = length(regexall("['\"\\\\]", var.rancher_registry_password)) == 0
    error_message = "rancher_registry_password must not contain quotes or backslashes."
  }
}

variable "ssh_user" {
  description = "SSH login user."
  type        = string
  default     = "ubuntu"
}

variable "host" {
  description = "Address of the machine reached over SSH."
  type        = string
}

variable "bastion_host" {
  description = "Optional SSH jump host (empty: direct)."
  type        = string
  default     = ""
}

variable "key_path" {
  description = "Private key used for SSH."
  type        = string
  default     = "~/.ssh/id_rsa"
}

variable "tk_operation" {
  description = "Which CLI operation runs this configuration (set by the executor through the root variable of the same name): apply runs the create-side data sources in full; destroy and read make them find-only and tolerant of hosts that are gone."
  type        = string
  default     = "apply"

  validation {
    condition     = contains(["apply", "destroy", "read"], var.tk_operation)
    error_message = "tk_operation must be apply, destroy or read."
  }
}

variable "tk_known_hosts" {
  description = "known_hosts lines of the cluster manager's pinned SSH host keys (set by the executor through the root variable of the same name, parallel/hostkeys.py)."
  type        = string
  default     = ""
}

variable "host_key" {
  description = "Pinned SSH host key of host (\"<type> <base64>\", set by the executor; empty: not pinned yet)."
  type        = string
  default     = ""
}

variable "bastion_host_key" {
  description = "Pinned SSH host key of bastion_host (set by the executor; empty: not pinned yet)."
  type        = string
  default     = ""
}

variable "node_cleanup" {
  description = "on destroy, take the host out of its cluster: uninstall rancher-system-agent and RKE2 (or the RKE1 containers) and remove their state, keeping the node tools and the container runtime (bare metal outlives its cluster; node/cleanup.py)"
  type        = bool
  default     = true
}

variable "gpu_product" {
  description = "Gpu product."
  type        = string
  default     = "MI355X"
}

variable "gpu_count" {
  description = "GPUs the node must expose"
  type        = number
  default     = 8
}

variable "gpu_burnin" {
  description = "quick | full | off"
  type        = string
  default     = "full"

  validation {
    condition     = contains(["quick", "full", "off"], var.gpu_burnin)
    error_message = "gpu_burnin must be quick, full or off."
  }
}

variable "rccl_env" {
  description = "RCCL / HSA environment for GPU pods"
  type        = map(string)
  default     = {}

  validation {
    condition     = alltrue([for k, v in var.rccl_env : length(regexall("^(NCCL|RCCL|HSA)_[A-Z0-9_]+$", k)) > 0 && length(regexall("(^|_)(PLUGIN|LIB|TOOLS|PATTERN|CONF|SCRIPT|DIR|PATH|[A-Z]*FILE)(_|$)", k)) == 0 && length(v) <= 256 && alltrue([for item in split(",", v) : length(regexall("^[A-Za-z0-9_.:=^+-]*(/[0-9]{1,3})?$", item)) > 0])])
    error_message = "rccl_env takes NCCL_*, RCCL_* and HSA_* settings whose values are comma lists of letters, digits and _ . : = ^ + - (an address range's /N allowed); settings that name a library, plugin, file, path or directory are not accepted."
  }
}

variable "rccl_min_busbw" {
  description = "node-level all-reduce bus bandwidth gate (GB/s)"
  type        = string
  default     = "0"

  validation {
    condition     = length(regexall("^[0-9]+([.][0-9]+)?$", var.rccl_min_busbw)) > 0
    error_message = "rccl_min_busbw must be a non-negative number (GB/s)."
  }
}

variable "gpu_link_min_frac" {
  description = "fail the node when a GPU pair's peer copy bandwidth is below this fraction of the node median"
  type        = string
  default     = "0.5"

  validation {
    condition     = length(regexall("^(0([.][0-9]+)?|1([.]0+)?|[.][0-9]+)$", var.gpu_link_min_frac)) > 0
    error_message = "gpu_link_min_frac must be a number between 0 and 1."
  }
}

variable "gpu_compute_partition" {
  description = "compute partition mode every GPU of the node must run in (spx | dpx | qpx | cpx); amd.com/gpu = gpu_count x partitions per GPU"
  type        = string
  default     = "spx"

  validation {
    condition     = contains(["spx", "dpx", "qpx", "cpx"], var.gpu_compute_partition)
    error_message = "gpu_compute_partition must be one of spx, dpx, qpx, cpx."
  }
}

variable "gpu_memory_partition" {
  description = "memory partition mode every GPU of the node must run in (nps1 | nps2)"
  type        = string
  default     = "nps1"

  validation {
    condition     = contains(["nps1", "nps2"], var.gpu_memory_partition)
    error_message = "gpu_memory_partition must be nps1 or nps2."
  }
}

variable "gpu_link_min_gbps" {
  description = "fail the node when a GPU pair's kernel-driven peer read is below this many GB/s (absolute floor: half of one xGMI link's ~76.8 GB/s one way)"
  type        = string
  default     = "38"

  validation {
    condition     = length(regexall("^[0-9]+([.][0-9]+)?$", var.gpu_link_min_gbps)) > 0
    error_message = "gpu_link_min_gbps must be a non-negative number (GB/s)."
  }
}

variable "gpu_host_tuning" {
  description = "host settings check (NUMA auto-balancing off, IOMMU passthrough): warn = labels and warnings; enforce = fail the node; off = not checked"
  type        = string
  default     = "warn"

  validation {
    condition     = contains(["warn", "enforce", "off"], var.gpu_host_tuning)
    error_message = "gpu_host_tuning must be warn, enforce or off."
  }
}

variable "gpu_health" {
  description = "GPU health policy (RAS counters): fail = an unhealthy GPU fails the node; taint = the node joins tainted amd.com/gpu-health=unhealthy:NoSchedule (no GPU pods); off = not checked"
  type        = string
  default     = "fail"

  validation {
    condition     = contains(["fail", "taint", "off"], var.gpu_health)
    error_message = "gpu_health must be fail, taint or off."
  }
}

variable "gpu_max_uncorrectable_ecc" {
  description = "uncorrectable ECC errors a GPU may have logged"
  type        = string
  default     = "0"

  validation {
    condition     = length(regexall("^[0-9]+$", var.gpu_max_uncorrectable_ecc)) > 0
    error_message = "gpu_max_uncorrectable_ecc must be a non-negative integer."
  }
}

variable "gpu_metrics_textfile" {
  description = "node_exporter textfile collector directory: write the GPU health metrics there (tk_gpu.prom) and refresh them every minute from a systemd timer (empty: off)"
  type        = string
  default     = ""

  validation {
    condition     = var.gpu_metrics_textfile == "" || (length(regexall("^/[A-Za-z0-9._/-]+$", var.gpu_metrics_textfile)) > 0 && length(regexall("/[.][.](/|$)", var.gpu_metrics_textfile)) == 0)
    error_message = "gpu_metrics_textfile must be empty or an absolute directory path."
  }
}

variable "gpu_max_retired_pages" {
  description = "retired VRAM pages a GPU may have (auto: the amdgpu driver's default threshold, one page per 100 MiB of VRAM)"
  type        = string
  default     = "auto"

  validation {
    condition     = var.gpu_max_retired_pages == "auto" || length(regexall("^[0-9]+$", var.gpu_max_retired_pages)) > 0
    error_message = "gpu_max_retired_pages must be a non-negative integer or auto."
  }
}

variable "rccl_slim" {
  description = "on: build a single-target (gfx950) copy of the node's librccl for faster cold communicator init, verify it with a one-rank all-reduce, and run rccl-ready on it while it matches the installed librccl (a modified vendor binary: off by default)"
  type        = string
  default     = "off"

  validation {
    condition     = contains(["on", "off"], var.rccl_slim)
    error_message = "rccl_slim must be on or off."
  }
}

variable "tk_prebuilt_tools" {
  description = "directory of prebuilt gfx950 node tools, each with its <tool>.sha256 source stamp, that the CLI stages (node/tools.py); empty: none uploaded, the node builds the tools with hipcc"
  type        = string
  default     = ""
}
