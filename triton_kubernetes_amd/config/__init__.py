from .context import Context, expand_home, file_exists, not_blank  # noqa: F401
from .prompt import NoPrompter, Prompter, ScriptedPrompter, TerminalPrompter  # noqa: F401
from .settings import Settings, load_config_file  # noqa: F401
